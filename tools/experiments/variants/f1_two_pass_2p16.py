# the two-pass F1 from 2^16 targets (cfg 2's 65,536) instead of 2^17
s = open("batch.hip").read()
a = "constexpr uint32_t kF1CoarseMinQ = 1u << 17;"
assert s.count(a) == 1
s = s.replace(a, "constexpr uint32_t kF1CoarseMinQ = 1u << 16;")
open("batch.hip", "w").write(s)
