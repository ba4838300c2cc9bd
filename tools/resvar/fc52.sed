filterbank.hip	s#constexpr int FR = 16, FC = 56;#constexpr int FR = 16, FC = 52;#
