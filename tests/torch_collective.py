"""keto_collective over torch.distributed (test / bench harness, not product): the object
partition's all-to-alls on a gloo process group (CPU tests, ranks sharing one GPU) or RCCL
(bench.py, one rank per GPU).  Host buffers in and out, as keto_collective specifies."""
import numpy as np
import torch
import torch.distributed as dist


class TorchCollective:
    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"

    def alltoall_u64(self, send: np.ndarray) -> np.ndarray:
        s = torch.from_numpy(send.astype(np.int64)).to(self.dev)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return r.cpu().numpy().astype(np.uint64)

    def alltoallv(self, send: np.ndarray, send_bytes, recv: np.ndarray, recv_bytes):
        s = torch.from_numpy(send).to(self.dev)
        r = torch.empty(int(sum(recv_bytes)), dtype=torch.uint8, device=self.dev)
        dist.all_to_all_single(r, s, [int(x) for x in recv_bytes], [int(x) for x in send_bytes], group=self.group)
        recv[:] = r.cpu().numpy()

    def allreduce_max_u64(self, v: int) -> int:
        t = torch.tensor([int(v)], dtype=torch.int64, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())
