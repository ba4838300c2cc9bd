wtp_internal.h	s#constexpr int RES_SIGMA_X100 = 400;#constexpr int RES_SIGMA_X100 = 350;#
