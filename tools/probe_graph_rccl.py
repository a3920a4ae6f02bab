"""Probe: can a torch.distributed (RCCL) all_reduce be captured inside a HIP graph on this stack?
World size 1 (the only size a 1-GPU box offers).  Prints the replayed results."""
import os

import torch
import torch.distributed as dist

os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
os.environ.setdefault('MASTER_PORT', '29531')
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
x = torch.ones(1 << 20, device='cuda')
dist.all_reduce(x)                       # eager warm-up (communicator init)
torch.cuda.synchronize()
print('eager ok', x[0].item(), flush=True)
g = torch.cuda.CUDAGraph()
src = torch.full([1 << 20], 3.0, device='cuda')
with torch.cuda.graph(g):
    y = src * 2
    w = dist.all_reduce(y, async_op=True)
    w.wait()
    z = y + 1
for v in [3.0, 5.0]:
    src.fill_(v)
    g.replay()
    torch.cuda.synchronize()
    print('replay', v, '->', z[0].item(), '(expect', 2 * v + 1, ')', flush=True)
dist.destroy_process_group()
print('probe done', flush=True)
