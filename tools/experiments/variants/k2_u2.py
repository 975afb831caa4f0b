# K2 with 2 uint4 of word 0 per lane per chunk (kClsU 3 -> 2)
s = open("table.hip").read()
a = "constexpr uint32_t kClsU = 3;"
assert s.count(a) == 1
s = s.replace(a, "constexpr uint32_t kClsU = 2;")
open("table.hip", "w").write(s)
