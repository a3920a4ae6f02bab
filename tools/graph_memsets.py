"""Inventory of the memset nodes inside the trainer's phase graphs (GPU diagnostic).

Builds the bench configuration, runs one eager step and one graph step (the captures), dumps each phase graph with
hipGraphDebugDotPrint (torch.cuda.CUDAGraph.debug_dump) and lists every memset node with the kernel nodes just
before and after it, so each can be traced to the op that issued it.

    python tools/graph_memsets.py [outdir]
"""
import argparse
import collections
import os
import re
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402

DEV = torch.device('cuda', 0)


def parse_dot(path):
    """(nodes: id -> label, edges: [(a, b)]) of a graph dump."""
    text = open(path, errors='replace').read()
    nodes, edges = {}, []
    for m in re.finditer(r'"?(\w+)"?\s*\[([^\]]*)\]', text):
        lab = re.search(r'label\s*=\s*"((?:[^"\\]|\\.)*)"', m.group(2)) or re.search(r'label\s*=\s*<(.*)>', m.group(2))
        nodes[m.group(1)] = lab.group(1) if lab else m.group(2)
    for m in re.finditer(r'"?(\w+)"?\s*->\s*"?(\w+)"?', text):
        edges.append((m.group(1), m.group(2)))
    return nodes, edges


def short(label):
    m = re.search(r'(?:name|func)[^\w]*([\w:<>~]+)', label)
    s = m.group(1) if m else label
    return s[:90]


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/graph_dump'
    os.makedirs(out, exist_ok=True)
    made = []

    class DbgGraph(torch.cuda.CUDAGraph):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.enable_debug_mode()
            made.append(self)

    torch.cuda.CUDAGraph = DbgGraph
    args = argparse.Namespace(res=256, batch_gpu=32, cbase=16384, img_channels=1, c_dim=2, map_depth=8,
                              fp16_dtype='fp16', phase_timing=False, deterministic='on')
    tr = bench.build(args, DEV, 0, 1)
    real, real_c = bench.make_inputs(args, DEV, 0)
    bench.one_step(tr, args, DEV, real, real_c)
    tr.graphs = True
    tr.batch_idx = 0
    bench.one_step(tr, args, DEV, real, real_c)
    torch.cuda.synchronize(DEV)
    names = list(tr._graphs.keys())
    print('phases captured:', names, 'graphs made:', len(made), flush=True)
    for name, st in tr._graphs.items():
        path = os.path.join(out, f'{name}.dot')
        st.graph.debug_dump(path)
        nodes, edges = parse_dot(path)
        succ, pred = collections.defaultdict(list), collections.defaultdict(list)
        for a, b in edges:
            succ[a].append(b)
            pred[b].append(a)
        kinds = collections.Counter()
        memsets = []
        for nid, lab in nodes.items():
            low = lab.lower()
            kind = 'memset' if 'memset' in low else ('memcpy' if 'memcpy' in low else ('kernel' if 'kernel' in low or
                                                                                      'func' in low else 'other'))
            kinds[kind] += 1
            if kind == 'memset':
                memsets.append(nid)
        print(f'== {name}: {len(nodes)} nodes {dict(kinds)}, {len(edges)} edges, '
              f'{sum(1 for n in nodes if len(pred[n]) > 1)} joins, {sum(1 for n in nodes if len(succ[n]) > 1)} forks',
              flush=True)
        for nid in memsets:
            lab = nodes[nid].replace('\\n', ' ')
            after = [short(nodes.get(s, s)) for s in succ[nid]]
            before = [short(nodes.get(p, p)) for p in pred[nid]]
            print(f'  memset {lab[:160]}\n     before {before[:2]}\n     after  {after[:2]}', flush=True)


if __name__ == '__main__':
    main()
