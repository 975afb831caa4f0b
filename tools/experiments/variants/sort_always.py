# sub-partitions always built prefix-sorted (the sort decision's threshold 0.10 -> 0): the
# prefix / shard shapes then take k_f2_direct too
s = open("api.hip").read()
a = "sort = 1.0 - std::exp(-qsub / (double)(1ull << lm)) > 0.10;"
assert s.count(a) == 1
s = s.replace(a, "sort = 1.0 - std::exp(-qsub / (double)(1ull << lm)) > 0.0;")
open("api.hip", "w").write(s)
