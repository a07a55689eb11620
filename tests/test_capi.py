"""CPU: liblgx.so loads and exports every entry point declared in include/lgx.h; argument checks
fail loudly without touching the GPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "lgx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(lgx_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for n in ["lgx_build_norm_adj", "lgx_propagate", "lgx_propagate_layer", "lgx_spmm_csr", "lgx_score_topk",
              "lgx_score_dense", "lgx_topk_rows", "lgx_foldout_metrics", "lgx_gather_scores", "lgx_version",
              "lgx_list_dot_reduce", "lgx_layer_epilogue"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from factors_of_serendipity_recommendation_amd import _lib
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"


def test_version_and_error_channel():
    from factors_of_serendipity_recommendation_amd import _lib
    L = _lib.lib()
    assert b"gfx950" in L.lgx_version()
    # k outside [1, 256] is rejected before any device work
    rc = L.lgx_topk_rows(None, 1, 10, 10, 0, None, None, None)
    assert rc != 0
    rc = L.lgx_topk_rows(ctypes.c_void_p(16), 1, 10, 10, 257, ctypes.c_void_p(16), None, None)
    assert rc == 3 and b"k=257" in L.lgx_last_error()
    with pytest.raises(RuntimeError, match="lgx_topk_rows"):
        _lib.check(rc, "lgx_topk_rows")


def test_lgx_csr_struct_layout_matches_header(tmp_path):
    """The ctypes mirrors of struct lgx_csr / lgx_plan have the header's size and field offsets
    (compiled from include/lgx.h with the host C compiler)."""
    import os
    import subprocess
    from factors_of_serendipity_recommendation_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fields = [f for f, _ in _lib.LgxCSR._fields_]
    pfields = [f for f, _ in _lib.LgxPlan._fields_]
    src = tmp_path / "layout.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"lgx.h\"\nint main(void){\n"
                   + 'printf("%zu %zu\\n", sizeof(lgx_csr), sizeof(lgx_plan));\n'
                   + "".join(f'printf("%zu\\n", offsetof(lgx_csr, {f}));\n' for f in fields)
                   + "".join(f'printf("%zu\\n", offsetof(lgx_plan, {f}));\n' for f in pfields)
                   + "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)])
    out = subprocess.check_output([str(exe)]).decode().split()
    assert int(out[0]) == ctypes.sizeof(_lib.LgxCSR) and int(out[1]) == ctypes.sizeof(_lib.LgxPlan)
    got = [int(x) for x in out[2:]]
    want = [getattr(_lib.LgxCSR, f).offset for f in fields] + [getattr(_lib.LgxPlan, f).offset for f in pfields]
    assert got == want


# the kernels bench.py times and the f4 label walk: their state stays in registers
HOT_KERNELS = ("spmm_segments", "spmm_fixup", "score_topk_bf16_lds", "score_topk_f32_lds", "score_topk_f32_pc",
               "score_topk_finalize",
               "strat_label_lds", "layer_epilogue", "score_dense_lds", "sum_slabs_kernel")


def test_hot_kernels_do_not_spill_to_scratch(tmp_path):
    """Host only: the hot gfx950 kernels of liblgx.so keep their state in registers -- no VGPR spills
    and no private (scratch) segment, read from the code object's metadata.  A spill in the scoring
    walk put a scratch reload on every top-k event (profiles/r03_score_lab_ws.txt: 54.79 -> 52.37 ms).
    The dense-score walk is held to 128 VGPRs where that fits without scratch (dense_waves_per_simd);
    its stores from a wave-uniform base removed the two spilled tile addresses of the fp32 d=256 walk."""
    import re
    import shutil
    import subprocess
    llvm = "/opt/rocm/lib/llvm/bin"
    if not (shutil.which("objcopy") and os.path.exists(f"{llvm}/clang-offload-bundler")):
        pytest.skip("objcopy / clang-offload-bundler not available")
    so = os.path.join(ROOT, "factors_of_serendipity_recommendation_amd", "liblgx.so")
    fat = tmp_path / "fat.bin"
    subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", so, str(fat)])
    # one offload bundle per translation unit, concatenated (and aligned) in the section
    blob = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
    assert len(starts) >= 5
    kernels = []
    for j, st in enumerate(starts):
        part, co = tmp_path / f"b{j}.bin", tmp_path / f"b{j}.o"
        part.write_bytes(blob[st:starts[j + 1] if j + 1 < len(starts) else len(blob)])
        subprocess.check_call([f"{llvm}/clang-offload-bundler", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}",
                               "--unbundle"])
        notes = subprocess.check_output([f"{llvm}/llvm-readelf", "--notes", str(co)]).decode()
        kernels += [b for b in notes.split("- .agpr_count:") if ".name:" in b]
    assert len(kernels) > 50
    bad = []
    for b in kernels:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", b).group(1))
        priv = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", b).group(1))
        if (spill or priv) and any(h in name for h in HOT_KERNELS):
            bad.append((name, spill, priv))
    assert sum(any(h in b for h in HOT_KERNELS) for b in kernels) >= 20
    assert not bad, bad


def test_ops_refuse_cpu_tensors():
    import torch
    import factors_of_serendipity_recommendation_amd as lgx
    with pytest.raises(RuntimeError, match="GPU only"):
        lgx.topk_rows(torch.zeros(2, 4), 1)
    with pytest.raises(RuntimeError, match="GPU only"):
        lgx.score_topk(torch.zeros(2, 8), torch.zeros(3, 8), 1)


def test_score_dense_rejects_catalogs_past_its_lane_offsets():
    """lgx_score_dense stores a tile's scores from a wave-uniform row base plus a 32-bit lane byte
    offset of up to (4 rows x n_items + 31) x 4 B: catalogs of 2^27 items or more are refused before
    any device work (host only: the pointers are never touched)."""
    from factors_of_serendipity_recommendation_amd import _lib
    L = _lib.lib()
    p = ctypes.c_void_p(16)
    assert L.lgx_score_dense(p, None, p, 4096, 1 << 27, 256, _lib.LGX_DTYPE_BF16, 0, p, None) == 3
    assert b"items is too many" in L.lgx_last_error()
    # empty calls stay no-ops
    assert L.lgx_score_dense(p, None, p, 0, 1 << 27, 256, _lib.LGX_DTYPE_BF16, 0, p, None) == 0


def test_new_entry_points_reject_bad_arguments_before_device_work():
    from factors_of_serendipity_recommendation_amd import _lib
    L = _lib.lib()
    p = ctypes.c_void_p(16)
    # unknown reduction
    assert L.lgx_list_dot_reduce(p, 64, 0, 1, p, p, p, p, 7, p, None) == 1
    # d beyond the kernel's register budget
    assert L.lgx_list_dot_reduce(p, 300, 0, 1, p, p, p, p, 0, p, None) == 3
    assert b"d=300" in L.lgx_last_error()
    # the epilogue has no PARTIAL mode, and needs its buffers
    assert L.lgx_layer_epilogue(p, 4, p, p, p, p, 64, 0, _lib.LGX_LAYER_PARTIAL, 1.0, None) == 1
    assert L.lgx_layer_epilogue(p, 4, None, p, p, p, 64, 0, _lib.LGX_LAYER_FIRST, 1.0, None) == 1


def test_sampler_rejects_bad_arguments_before_device_work():
    from factors_of_serendipity_recommendation_amd import _lib
    L = _lib.lib()
    p = ctypes.c_void_p(16)
    # no user list and no rows per user
    assert L.lgx_sample_bpr(p, p, 10, 100, None, 10, 0, 1, 1, p, None) == 1
    # more rows than users * per_user
    assert L.lgx_sample_bpr(p, p, 10, 100, None, 101, 10, 1, 1, p, None) == 1
    # empty catalog
    assert L.lgx_sample_bpr(p, p, 10, 0, None, 10, 1, 1, 1, p, None) == 1


def test_stratification_rejects_bad_arguments_before_device_work():
    from factors_of_serendipity_recommendation_amd import _lib
    L = _lib.lib()
    p = ctypes.c_void_p(16)
    assert L.lgx_strat_labels(p, 1, 10, 0.0, 0.0, 10, None, None, p, p, None) == 1  # inter must be > 0
    assert L.lgx_strat_labels(p, 1, 10, 0.0, 0.5, 40, None, None, p, p, None) == 1  # too many folds
    assert L.lgx_strat_select(p, 1, 10, p, 11, p, 1, p, 2048, p, None) == 3         # > 1024 per user


@pytest.mark.parametrize("mn,mx,num_fold", [(-0.731, 1.42, 10), (0.0, 3.0, 10), (-4.5, 2.25, 7), (-1e-3, 1e-3, 10),
                                            (-20.0, 35.5, 31), (-12.97, 9.34, 10)])
def test_strat_thresholds_reproduce_float16_labels(mn, mx, num_fold):
    """Host only: lgx_strat_thresholds' step function == numpy's float16 label arithmetic
    (recommend.py:375-381: (f16(s) - min16) / inter16, floored, the division in the float16 loop)
    on random scores, on every threshold and on its f32 neighbours.  inter16 as the reference's
    pinned numpy forms it (legacy promotion, recommend.legacy_float16_bounds)."""
    import numpy as np
    from factors_of_serendipity_recommendation_amd import _lib, recommend
    L = _lib.lib()
    m, i16 = recommend.legacy_float16_bounds(mx, mn, num_fold, 0.1)
    min16, inter16 = np.float16(m), np.float16(i16)
    thr = (ctypes.c_float * num_fold)()
    assert L.lgx_strat_thresholds(float(min16), float(inter16), num_fold, thr) == 0
    t = np.array(thr[:], dtype=np.float32)
    assert (np.diff(t) >= 0).all()
    rng = np.random.default_rng(num_fold)
    fin = t[np.isfinite(t)]
    s = np.concatenate([rng.uniform(mn - 1.0, mx + 1.0, 200_000).astype(np.float32), fin,
                        np.nextafter(fin, -np.inf, dtype=np.float32), np.nextafter(fin, np.inf, dtype=np.float32),
                        np.array([mn, mx, -1e30, 1e30], dtype=np.float32)])
    with np.errstate(over="ignore", invalid="ignore"):
        q = np.floor((s.astype(np.float16) - min16) / inter16).astype(np.float64)
    ref = np.clip(np.nan_to_num(q, nan=num_fold, posinf=num_fold, neginf=0), 0, num_fold).astype(np.int64)
    got = (s[:, None] >= t[None, :]).sum(1)
    assert np.array_equal(got, ref)


def test_score_topk_plan_seeds_large_full_sweeps():
    """Host only (lgx_score_topk_plan): the full-sweep LDS plan is swept in seeded stages once the
    catalog reaches 262 144 items; smaller catalogs and catalog-split launches run as one launch."""
    import torch
    from factors_of_serendipity_recommendation_amd import ops
    big = ops.score_topk_plan(1_000_000, 1_000_000, 256, torch.bfloat16, 20)
    assert big.split("; ")[0].endswith("full-sweep (seeded in stages) (score floors) n_splits=1 utiles=3840"), big
    assert "seeded" not in big.split("; ")[1]
    assert "seeded" in ops.score_topk_plan(65536, 262_144, 256, torch.bfloat16, 20)
    assert "seeded" not in ops.score_topk_plan(65536, 262_143, 256, torch.bfloat16, 20)
    assert "seeded" not in ops.score_topk_plan(4096, 1_000_000, 256, torch.bfloat16, 20)
    f32 = ops.score_topk_plan(262_144, 1_000_000, 256, torch.float32, 20)
    assert f32.endswith("full-sweep (seeded in stages) n_splits=1 utiles=2048"), f32
