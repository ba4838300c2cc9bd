kernels.hip	s/auto key = \[\&\](float v) { atomicAdd(\&wl.h\[key_bin(abs_key(v))\], 1u); };/auto key = [\&](float v) { if (v == 12345.0f) wl.h[0] = 1u; };/
