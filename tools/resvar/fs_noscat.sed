kernels.hip	s/            if ((keep >> p) \& 1u) put(w\[p\]);/            if (((keep >> p) \& 1u) \&\& w[p] == 7u) put(w[p]);/
