kernels.hip	s/for (int k = 1; k <= sg.L; ++k) {$/for (int k = 1; k <= 1; ++k) {/
