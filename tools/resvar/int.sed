filterbank.hip	s#raw_buffer_load_b32(rP, vo, s\([VHD]\), 0))#raw_buffer_load_b32(rP, vo, s\1, 2))#
