filterbank.hip	s#raw_buffer_store_b32(__float_as_uint(\(hg.x\|lw.y\|hg.y\)), rP, \(voff\|vo\), \(.*\), 0);#raw_buffer_store_b32(__float_as_uint(\1), rP, \2, \3, 2);#
