wtp_internal.h	s#constexpr bool RES_LASTSEL = true;#constexpr bool RES_LASTSEL = false;#
