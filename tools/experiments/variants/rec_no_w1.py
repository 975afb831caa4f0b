# timing only (results wrong): the record form's fast path without the word-1 loads
s = open("batch.hip").read()
a = "                            w1[r] = a.planes[a.stride + res[r]];\n"
assert s.count(a) == 1
s = s.replace(a, "                            w1[r] = res[r] * 3u;\n")
open("batch.hip", "w").write(s)
