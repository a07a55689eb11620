"""Development: cycle breakdown of the LDS scoring walk from the stamped lab build
(tools/make_stats_lab.py -> tools/_ab/lab/.../liblgx.so).  Per call: the walk's phases in shader
cycles per (wave, tile) -- refill staging, the late waves' epilogue, the MFMA issue (compute), the
early waves' epilogue, the vmcnt wait + barrier -- and how a wave's tiles split between the fast
path, the deferred path and the full (regroup + exact) path.

  python tools/score_stats.py [--only eval|c5]
"""
import ctypes
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
from factors_of_serendipity_recommendation_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("LGX_LAB_LIB") or os.path.join(ROOT, "tools", "_ab", "lab", "factors_of_serendipity_recommendation_amd",
                                                               "liblgx.so")
_lib._lib = None
_lib.ALLOW_MISSING = True
import make_stats_lab  # noqa: E402
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import evaluator, ops  # noqa: E402

L = _lib.lib()
L.lgx_lab_stats.restype = ctypes.c_int
L.lgx_lab_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
ONLY = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None


def stats(fn, label):
    fn()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 32)()
    L.lgx_lab_stats(buf, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    L.lgx_lab_stats(buf, 1)
    v = dict(zip(make_stats_lab.FIELDS, list(buf)[:len(make_stats_lab.FIELDS)]))
    wt = max(1, v["tiles"])
    per = {k: v[k] / wt for k in ("cyc_loop", "cyc_stage", "cyc_epi_late", "cyc_compute", "cyc_epi_early", "cyc_wait")}
    frac = {k: v[k] / wt for k in ("n_fast", "n_event_tiles", "n_defer", "n_full")}
    full_cyc = v["cyc_full"] / max(1, v["n_full"])
    det = v["cyc_detect"] / wt
    dfr = v["cyc_defer"] / max(1, v["n_defer"])
    print(f"{label}: {e0.elapsed_time(e1):.2f} ms (stamped), {v['waves']} waves, {v['tiles'] / max(1, v['waves']):.0f} tiles/wave", flush=True)
    print("   cycles per wave-tile: " + ", ".join(f"{k[4:]} {x:.0f}" for k, x in per.items()), flush=True)
    print("   per wave-tile: " + ", ".join(f"{k[2:]} {x:.3f}" for k, x in frac.items())
          + f"; cycles per full path {full_cyc:.0f}; flush {v['cyc_flush'] / max(1, v['waves']):.0f} per wave; "
            f"detect (incl. the MFMA results' wait) {det:.0f} per wave-tile; deferred path {dfr:.0f} per deferral", flush=True)
    if v.get("pc_waves"):
        print(f"   producer/consumer: producers per tile: score writes {v['cyc_pc_write'] / wt:.0f}, refill + MFMA issue "
              f"{v['cyc_pc_compute'] / wt:.0f}, vmcnt {v['cyc_pc_vm'] / wt:.0f}, barrier {v['cyc_pc_pwait'] / wt:.0f}; "
              f"consumers: epilogue {per['cyc_epi_early']:.0f}, barrier {v['cyc_pc_cwait'] / wt:.0f}", flush=True)
    nf = max(1, v["n_full"])
    print(f"   per full path: drop_masked {v['cyc_dropmasked'] / nf:.0f}, drain inserts {v['cyc_drain_ins'] / nf:.0f}, "
          f"direct inserts {v['cyc_insert_now'] / nf:.0f} cycles (flush included); unbounded {v['n_unbounded'] / nf:.3f}; "
          f"rescans per lane {v['n_rescan'] / nf / 64:.1f}, drain steps {v['n_drain_steps'] / nf:.1f}", flush=True)


if ONLY in (None, "eval"):
    import bench_rows as br
    from factors_of_serendipity_recommendation_amd.model import LightGCN
    with tempfile.TemporaryDirectory() as tmp:
        for name in ("gowalla", "amazon"):
            cfg = br.CONFIGS[name]
            ds = br._eval_dataset(cfg, tmp)
            conf = {"latent_dim_rec": cfg.d, "lightGCN_n_layers": cfg.K, "keep_prob": 0.6, "A_split": False,
                    "pretrain": 0, "dropout": 0}
            torch.manual_seed(0)
            model = LightGCN(conf, ds).to("cuda").eval()
            with torch.no_grad():
                U, I = model.computer()
            tl = evaluator._TestLists.get(ds, I.shape[0], U.device)
            r = tl.route(I.shape[0], 20, cfg.d)
            rows, mask = (r.light_rows, r.light_mask) if r.n_heavy else (tl.rows, tl.mask)
            plan = ops.score_topk_plan(rows.numel(), I.shape[0], cfg.d, torch.float32, 20)
            stats(lambda: ops.score_topk(U, I, 20, user_rows=rows, mask=mask, mask_value=-1024.0, apply_sigmoid=True),
                  f"{name} propagated, light users, masked [{plan}]")
            stats(lambda: ops.score_topk(U, I, 20, user_rows=rows), f"{name} propagated, light users, unmasked")
            stats(lambda: ops.score_topk(U, I, 1, user_rows=rows), f"{name} propagated, light users, top-1")
            Qr = lgx.fill_normal((rows.numel(), cfg.d), 0.1, 7)
            Ir = lgx.fill_normal((I.shape[0], cfg.d), 0.1, 8)
            stats(lambda: ops.score_topk(Qr, Ir, 20), f"{name} random tables, unmasked")
            del model, ds
            torch.cuda.empty_cache()

if ONLY in (None, "c5"):
    d, n_items, B = 256, 1_000_000, 262_144
    items = lgx.fill_normal((n_items, d), 1.0 / 16, 4242, dtype=torch.bfloat16)
    Q = lgx.fill_normal((B, d), 1.0 / 16, 777, dtype=torch.bfloat16)
    g = torch.Generator(device="cuda")
    g.manual_seed(99)
    pos = torch.randint(0, n_items, (B, 50), device="cuda", generator=g).sort(dim=1).values
    mask = (torch.arange(0, B + 1, device="cuda", dtype=torch.int64) * 50, pos.reshape(-1).to(torch.int32))
    stats(lambda: ops.score_topk(Q, items, 20, mask=mask), "C5 bf16 262144 x 1M, masked (every stage and launch summed)")
