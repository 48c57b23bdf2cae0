"""Probe: RCCL communicator init inside the extension vs torch's nccl backend
(one rank).  usage: python tools/probes/rccl_probe.py torch|cek"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

which = sys.argv[1]
if which == "torch":
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29555", RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    t = torch.ones(16, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print("torch nccl ok", t.sum().item(), flush=True)
    dist.destroy_process_group()
else:
    from cekirdekler_amd._native import cek
    uid = cek.RcclComm.unique_id()
    print("unique id bytes", len(uid), flush=True)
    c = cek.RcclComm(uid, 0, 1, 0)
    print("cek comm ok", c.rank, c.world, flush=True)
