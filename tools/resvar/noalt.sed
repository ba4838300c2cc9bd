api.hip	s#constexpr bool FB_ALT_ORDER = true;#constexpr bool FB_ALT_ORDER = false;#
