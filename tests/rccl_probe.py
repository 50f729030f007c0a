"""Child-process probe for tests/test_gpu_rccl.py (not a test module): one rank of an RCCL ("nccl")
process group on cuda:0 runs every shard.py collective on device tensors and prints one JSON line.
Run as a child so that the RCCL communicator lives and dies with its own process."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fancy_gym_crowd_amd import shard  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["FGX_PROBE_PORT"], rank=0, world_size=1,
                        device_id=dev)
ret = torch.arange(1000, dtype=torch.float64, device=dev) * 0.5
g = shard.gather_returns(ret)
out = {"backend": dist.get_backend(), "world": dist.get_world_size(),
       "gather_ok": bool(torch.equal(g, ret)), "gather_device": str(g.device),
       "max": shard.max_over_ranks(3.25, dev), "sum": shard.sum_over_ranks(7, dev),
       "ints": shard.gather_ints([1, 2, 3], dev), "floats": shard.gather_floats([0.5, 1.5], dev)}
dist.barrier()
dist.destroy_process_group()
print(json.dumps(out), flush=True)
