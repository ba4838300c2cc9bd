filterbank.hip	s#    constexpr int HALF = fwd_lhh(NCc);#    constexpr int HALF = (NCc + 1) / 2;#
filterbank.hip	s#    static_assert(HALF % 16 == 8 \&\& HALF >= (NCc + 1) / 2, "LH half pitch");##
filterbank.hip	s#    auto lhi = \[\&\](int o, int cc) { return o \* (2 \* HALF) + (cc \& 1) \* HALF + (cc >> 1); };#    auto lhi = [\&](int o, int cc) { return o * NCc + (cc \& 1) * HALF + (cc >> 1); };#
