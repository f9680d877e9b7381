"""Run by tests/test_gpu_dist.py in a fresh process: the RCCL ("nccl") process group at world
size 1 on a TCP store on loopback, created before any other HIP use of the process, and the
bench's two collectives (mpcx/dist.py all_gather_stats, max_over_ranks) on cuda tensors through
it.  Prints one JSON line with what it checked."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))

import numpy as np  # noqa: E402

with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
os.environ.update({"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                   "MASTER_PORT": str(port)})

from mpcx import dist as mdist  # noqa: E402

rank, world = mdist.init("nccl", always=True)  # before any other HIP call of this process
import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

torch.cuda.set_device(0)
assert tdist.is_initialized() and tdist.get_backend() == "nccl" and (rank, world) == (0, 1)
rng = np.random.default_rng(5)
S = rng.standard_normal((4096, len(mdist.STAT_FIELDS)))
S_all = mdist.all_gather_stats(S, device=torch.device("cuda", 0))
assert S_all.shape == S.shape and np.array_equal(S_all, S)
t = mdist.max_over_ranks(3.25, device=torch.device("cuda", 0))
assert t == 3.25
# the collective really moved device memory: an all_gather of a cuda tensor into cuda outputs
x = torch.arange(1000, dtype=torch.float64, device="cuda")
out = [torch.empty_like(x)]
tdist.all_gather(out, x)
torch.cuda.synchronize()
assert out[0].is_cuda and torch.equal(out[0], x)
print(json.dumps({"backend": tdist.get_backend(), "world": world, "stats_shape": list(S_all.shape),
                  "max_over_ranks": t, "nccl_version": str(torch.cuda.nccl.version())}))
tdist.destroy_process_group()
