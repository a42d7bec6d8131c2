"""Device footprint of one rank's resident partition (the distributed frontier's snapshot) at a
config-5 scale: rank R of W of the Drive forest x S, built alone on the box's GPU with a
stand-in collective that answers every exchange with this rank's own data (the job-wide OR of
relation flags is then this rank's: the footprint is the same).  KETO_PART_VERBOSE prints the
snapshot's nodes, bytes and build time; hipMemGetInfo before / after."""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "djy-keto_amd")]


class SelfCollective:
    def __init__(self, rank, world):
        self.rank, self.world, self.device_buffers = rank, world, False

    def alltoall_u64(self, send):
        return np.array([send[self.rank]] * self.world, dtype=np.uint64)

    def alltoallv(self, send, send_bytes, recv, recv_bytes):
        off = sum(send_bytes[:self.rank])
        mine = send[off:off + send_bytes[self.rank]]
        o = 0
        for b in recv_bytes:
            recv[o:o + b] = mine[:b]
            o += b

    def allreduce_max_u64(self, v):
        return v


def free_gib():
    hip = ctypes.CDLL("libamdhip64.so")
    fr, tot = ctypes.c_size_t(), ctypes.c_size_t()
    hip.hipMemGetInfo(ctypes.byref(fr), ctypes.byref(tot))
    return fr.value / 2**30, tot.value / 2**30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=40)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args()
    os.environ["KETO_PART_VERBOSE"] = "1"
    from keto_mi355x import partition, synth
    wl = synth.drive_scaled(a.scale, materialize=False)
    t0 = time.perf_counter()
    part = synth.drive_partition(wl, a.world, a.rank)
    t1 = time.perf_counter()
    f0 = free_gib()
    print(f"partition {a.rank}/{a.world} of x{a.scale}: {len(part)} tuples, generated {t1 - t0:.1f} s; free {f0[0]:.1f} of {f0[1]:.0f} GiB",
          flush=True)
    eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids, part,
                                      max_read_depth=wl.max_depth, max_read_width=wl.max_width,
                                      collective=SelfCollective(a.rank, a.world))
    del part
    f1 = free_gib()
    print(f"built in {time.perf_counter() - t1:.1f} s; free {f1[0]:.1f} GiB (held {f0[0] - f1[0]:.1f} GiB)", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
