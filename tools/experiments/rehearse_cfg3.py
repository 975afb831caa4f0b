"""Rehearse bench.py's N > 1 cfg-3 leg (cfg3_multi_leg: 10^9 ids, 2^20 targets, broadcast and
prefix routes) on ONE GPU as a world of 1 over RCCL, so that the code path the driver's
multi-GPU run takes (sub-partitioned K6 in record mode, all-gather, K3 merge; prefix shards)
is exercised end to end before that run.  Also re-checks the merged results of the broadcast
route on a target sample against the library's own K1 scan over the same ids.
usage: python tools/experiments/rehearse_cfg3.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
import opendht_amd  # noqa: E402


class A:
    seed = 2024
    k = 8
    no_cpu = False


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    L = opendht_amd.lib()
    out = bench.cfg3_multi_leg(A(), L, dev, stream.cuda_stream, stream, 1, 0)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
