kernels.hip	s/            v\[j\] = x\[(int64_t)(i \/ PS) \* sg.C + (i % PS)\];/            v[j] = (float)(i \& 7) * (float)(x == nullptr);/
