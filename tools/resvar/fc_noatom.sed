filterbank.hip	s/            if (f_below) atomicAdd(\&sst->below\[sh8\], (unsigned long long)f_below);//
filterbank.hip	s/            if (f_eq) atomicAdd(\&sst->eq_lo\[sh8\], (unsigned long long)f_eq);//
filterbank.hip	s/            if (mx) atomicMax(\&sst->maxkey\[sh8\], mx);//
