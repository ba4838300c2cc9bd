kernels.hip	s#__builtin_nontemporal_store(yv, reinterpret_cast<f4v\*>(q4 + it \* CT + tid));#*reinterpret_cast<f4v*>(q4 + it * CT + tid) = yv;#
