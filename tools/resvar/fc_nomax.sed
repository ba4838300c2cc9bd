filterbank.hip	s/        f_mx = (ok \&\& k > f_mx) ? k : f_mx;//
