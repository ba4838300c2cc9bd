wtp_internal.h	s#constexpr int RES_LATE_PCT = 60;#constexpr int RES_LATE_PCT = 0;#
