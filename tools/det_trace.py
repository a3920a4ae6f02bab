"""det_sum calls of the training step (GPU diagnostic): run under SG2_DET_TRACE=1 (det.hip prints one line per call:
G, n, S, chunks K) and rocprofv3 --kernel-trace; tools/det_trace_join.py pairs the lines with the det_sum dispatches
in order and sums the time per call shape over one 16-step cycle (eager: the graphs replay the same launches).
    SG2_DET_TRACE=1 rocprofv3 --kernel-trace --output-format csv -d OUT -- python tools/det_trace.py 2> calls.txt"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402

sys.argv = [sys.argv[0], '--graphs', 'off', '--no-cpu-baseline']
args = bench.parse()
dev = torch.device('cuda', 0)
tr = bench.build(args, dev, 0, 1)
real, real_c = bench.make_inputs(args, dev, 0)
for _ in range(2):
    bench.one_step(tr, args, dev, real, real_c)
torch.cuda.synchronize()
sys.stderr.write('CYCLE_BEGIN\n')
sys.stderr.flush()
for _ in range(16):
    bench.one_step(tr, args, dev, real, real_c)
torch.cuda.synchronize()
sys.stderr.write('CYCLE_END\n')
sys.stderr.flush()
