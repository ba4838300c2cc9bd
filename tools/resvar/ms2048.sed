wtp_internal.h	s#constexpr int RES_MS = 4096;#constexpr int RES_MS = 2048;#
