# timing only (results wrong): the record form's fast-path row written as 2 uint4 (the index form's
# store count) instead of 6
s = open("batch.hip").read()
a = "for (int r = 0; r < 3 * K; r += 4)\n                                *reinterpret_cast<uint4*>(ro + r)"
assert s.count(a) == 1
s = s.replace(a, "for (int r = 0; r < 8; r += 4)\n                                *reinterpret_cast<uint4*>(ro + r)")
open("batch.hip", "w").write(s)
