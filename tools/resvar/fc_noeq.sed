filterbank.hip	s/        f_eq += (uint32_t)__popcll(__ballot(ok \&\& k == skl));//
