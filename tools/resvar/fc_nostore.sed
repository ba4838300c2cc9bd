filterbank.hip	s/            if (in \&\& pos < (uint32_t)FSL_KEYS) wslot\[1 + pos\] = k;//
