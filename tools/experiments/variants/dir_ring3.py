# k_f2_direct with a ring of 3 sub-steps (48 KB in flight per CU) instead of kF2Ring = 2
s = open("batch.hip").read()
i = s.index("void k_f2_direct(F2Args a)")
j = s.index("// ---- candidate order ----")
body = s[i:j]
assert body.count("kF2Ring") == 5
body = body.replace("kF2Ring", "kDirRingV")
s = s[:i] + body + s[j:]
s = s.replace("constexpr uint32_t kDirParts = 4096;", "constexpr uint32_t kDirParts = 4096;\nconstexpr uint32_t kDirRingV = 3;")
open("batch.hip", "w").write(s)
