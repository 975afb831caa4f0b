"""Crawl replay: tools/dhtscanner.cpp's network scan driven by batched iterative searches.

The scanner (reference tools/dhtscanner.cpp:49-72, main :110-118) starts at the hash with
only bit 159 set, depth 0.  Each step runs a `get` (an iterative search) on its hash; when
it completes with the search's nodes (Search::getNodes, src/search.h:724-732: every
SearchNode, bad ones included) it
  * adds them to the set of all nodes found,
  * computes bdepth = commonBits(first, last) of the nodes in id order (0 for one node) and
    target_depth = min(8, bdepth + 6) (:59-60),
  * recurses on its hash with bit b set, at depth b + 1, for b in [cur_depth, target_depth)
    (:62-66).
A step's children depend only on its own search, so the steps are run generation by
generation, each generation as ONE batched search call (libdhtgpu's search kernel, or the
oracle restatement in the tests) -- the set of steps and of nodes found is the one the
reference's callback recursion produces.
"""
import numpy as np

ROOT_BIT = 159
MAX_DEPTH = 8
DEPTH_SLACK = 6


def set_bit(h, b):
    """InfoHash::setBit(nbit, true) (include/opendht/infohash.h:196-210): MSB-first bit numbering."""
    h = h.copy()
    h[b // 8] |= 0x80 >> (b % 8)
    return h


def common_bits(a, b):
    """InfoHash::commonBits (include/opendht/infohash.h:154-176)."""
    x = int.from_bytes(bytes(a), "big") ^ int.from_bytes(bytes(b), "big")
    return 160 - x.bit_length()


def crawl(search, node_ids, scanner_node, max_rounds=64):
    """Run the scan.  search(targets (m,20) uint8, searchers (m,) uint32, max_rounds) ->
    (idx (m,64), flags, len, rounds, queries); node_ids(indices) -> (k,20) ids.
    Returns a dict: steps, generations, nodes found (sorted indices), queries, rounds."""
    root = set_bit(np.zeros(20, np.uint8), ROOT_BIT)
    gen = [(root, 0)]
    found = set()
    steps = queries = rounds = generations = 0
    per_gen = []
    while gen:
        generations += 1
        tg = np.stack([h for h, _ in gen])
        idx, fl, ln, rd, qs = search(tg, np.full(len(gen), scanner_node, np.uint32), max_rounds)
        steps += len(gen)
        queries += int(qs.sum())
        rounds += int(rd.sum())
        per_gen.append((len(gen), int(qs.sum()), int(rd.max()) if len(gen) else 0))
        nxt = []
        for i, (h, depth) in enumerate(gen):
            nodes = [int(x) for x in idx[i, : ln[i]]]
            found.update(nodes)
            if not nodes:
                continue
            ids = node_ids(np.array(nodes, dtype=np.int64))
            order = np.lexsort(ids.T[::-1])
            first, last = ids[order[0]], ids[order[-1]]
            bdepth = 0 if len(nodes) == 1 else common_bits(first, last)
            target = min(MAX_DEPTH, bdepth + DEPTH_SLACK)
            for b in range(depth, target):
                nxt.append((set_bit(h, b), b + 1))
        gen = nxt
    return {"steps": steps, "generations": generations, "found": np.array(sorted(found), dtype=np.uint32),
            "queries": queries, "rounds": rounds, "per_generation": per_gen}
