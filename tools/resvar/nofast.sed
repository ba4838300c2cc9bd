filterbank.hip	s#constexpr bool FB_FAST_INTERIOR = true;#constexpr bool FB_FAST_INTERIOR = false;#
