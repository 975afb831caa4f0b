# cfg 2 through the sub-partition path (2 prefix-sorted sub-partitions of 2^23, k_f2_direct) instead
# of the one-set K6: the stage-free F2 leaves its CU's LDS to F3
s = open("api.hip").read()
a = "    return c->n > (1ull << 24) && !batch_supported(c->n, q, k, c->num_cus) && q <= (1u << 22);"
assert s.count(a) == 1
s = s.replace(a, "    return (c->n >= (1ull << 23) && q >= 32768 && q <= (1u << 22)) ||\n"
                 "           (c->n > (1ull << 24) && !batch_supported(c->n, q, k, c->num_cus) && q <= (1u << 22));")
open("api.hip", "w").write(s)
