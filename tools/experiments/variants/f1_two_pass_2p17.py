# the two-pass F1 from 2^17 targets (the cfg-3 prefix / shard shapes) instead of 2^18
s = open("batch.hip").read()
a = "constexpr uint32_t kF1CoarseMinQ = 1u << 18;"
assert s.count(a) == 1
s = s.replace(a, "constexpr uint32_t kF1CoarseMinQ = 1u << 17;")
open("batch.hip", "w").write(s)
