kernels.hip	s#        if (FULL) load_chunk<IT, CT>(p, v);#        if (FULL) load_chunk<IT, CT, true>(p, v);#
kernels.hip	s#        else load_chunk_ragged<IT, CT>(p, len, v);#        else load_chunk_ragged<IT, CT, true>(p, len, v);#
