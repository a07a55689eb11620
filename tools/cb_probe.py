"""Development probe: the product's column-blocked layer (graph.CSRGraph.col_blocks) at C4, f32 and
bf16, by block count; each line the PLAIN / STACK layer time (HIP events, min of reps)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import _lib, ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_graph  # noqa: E402


def timed(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts)


cfg = CONFIGS["synth10m"]
U, I, d = cfg.n_users, cfg.n_items, cfg.d
A = synth_graph(cfg, seed=2020, device="cuda")
N = U + I
for dt, es in ((torch.float32, 4), (torch.bfloat16, 2)):
    E0 = lgx.fill_normal((N, d), 0.1, 2020, dtype=dt)
    Y = torch.empty((N, d), dtype=dt, device="cuda")
    for nb in (0, 4, 8, 13, 16, 24):
        if nb == 0:
            A.col_blocking = False
        else:
            A.col_blocking = True
            A.col_block_slice = -(-U * d * es // nb)
            assert A.col_block_count(d, es) == nb
        ms = timed(lambda: ops.propagate_layer(A, E0, _lib.LGX_LAYER_PLAIN, Y=Y))
        print(f"{'f32' if es == 4 else 'bf16'} PLAIN layer, item rows in {nb:2d} column blocks: {ms:8.3f} ms", flush=True)
    del E0, Y
    torch.cuda.empty_cache()
print("probe done", flush=True)
