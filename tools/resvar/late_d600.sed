kernels.hip	s#^    WTP_RPROBE(0);$#    WTP_RPROBE(0);\n    const uint64_t t_beg_ = wall_ticks();#
kernels.hip	s#        if (sd.flags \& SEG_LATE) __syncthreads(); /\* block-uniform \*/#        if (sd.flags \& SEG_LATE) { __syncthreads(); while (wall_ticks() - t_beg_ < 600) __builtin_amdgcn_s_sleep(4); }#
