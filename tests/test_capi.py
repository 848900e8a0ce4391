"""The C-ABI library builds, loads and exports every symbol of include/vqgnn.h
(no compute calls: no GPU here)."""
import os
import re

import vq_gnn_amd._lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "vqgnn.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vqgnn_\w+)\s*\(", text)))


def test_library_exports_header_symbols():
    h = L.lib()
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(h, s), f"missing export {s}"
        assert s in L.SIGNATURES, f"no ctypes signature for {s}"
    assert set(L.SIGNATURES) == set(syms)


def test_version_and_error_text():
    h = L.lib()
    assert h.vqgnn_version() >= 100
    assert h.vqgnn_last_error() == b""


def test_host_only_workspace_queries():
    h = L.lib()
    assert h.vqgnn_bn_stats_workspace(84670, 128) > 0
    assert h.vqgnn_vq_assign_workspace(84670, 32, 256, 8) >= 256       # fused EMA
    assert h.vqgnn_vq_assign_workspace(30000, 64, 4096, 8) >= 64 * 30000 * 4  # idx scratch
    assert 1 <= h.vqgnn_vq_ema_parts(84670, 32, 256, 8) <= 64
    import ctypes
    sf, sg = ctypes.c_int32(), ctypes.c_int32()
    h.vqgnn_vq_stat_shifts(84670, 1.0, ctypes.byref(sf), ctypes.byref(sg))
    # |z| <= sqrt(84670) ~ 291 < 2^9  ->  2^(30-9) keeps a row inside int32
    assert (sf.value, sg.value) == (21, 21)
    h.vqgnn_vq_stat_shifts(84670, 2.0 ** -10, ctypes.byref(sf), ctypes.byref(sg))
    assert (sf.value, sg.value) == (21, 31)
    assert h.vqgnn_spmm_task_workspace(2_000_000, 64, 128) > 0
    assert h.vqgnn_spmm_task_size(2_000_000, 64, 128000) == 5 * 31250 + 1 + 128000


def test_invalid_arguments_rejected_without_device():
    # argument validation happens before any launch
    h = L.lib()
    rc = h.vqgnn_vq_assign(None, 0, None, 0, 10, 1, 4, 16, 6, None, 1.0, None, 8, 128,
                           None, None, 0, None, None, 0, 0, None, None)
    assert rc == 1
    assert b"null" in h.vqgnn_last_error() or b"W" in h.vqgnn_last_error()
    # dummy non-null addresses: validation rejects F before any pointer is used
    rc = h.vqgnn_spmm_task(16, 4, 4, 0, 0, None, 4, None, 0, 6, 16, 4, 16, None, 64, 0, 0,
                           None, None)
    assert rc == 1 and b"multiple of 4" in h.vqgnn_last_error()
    rc = h.vqgnn_spmm_task(None, 4, 4, 0, 0, None, 4, None, 0, 8, None, 8, None, None, 64, 0, 0,
                           None, None)
    assert rc == 1 and b"null" in h.vqgnn_last_error()
    # the plan's edge count is bounded by its int32 task starts
    rc = h.vqgnn_spmm_task_plan(16, 16, None, 4, 1 << 31, 64, 16, 16, 16, None)
    assert rc == 1 and b"bad arguments" in h.vqgnn_last_error()
    # the code exchange's stamp epochs start at 1
    rc = h.vqgnn_scatter_wire(16, 4, 8, 256, 16, 0, 10, 16, 8, None)
    assert rc == 1 and b"epoch" in h.vqgnn_last_error()


def test_codebook_reads_bounded_by_its_branch_count():
    """VERDICT r04 (GPU fault): the gather and the codebook-source SpMM take
    the codebook's branch count and reject a call that would read past it --
    before any launch, so dummy device addresses never get dereferenced."""
    h = L.lib()
    # gather: 35 code columns against a 32-branch [32, 256, 8] codebook
    rc = h.vqgnn_gather_codewords(16, 100, 200, 16, 35, 1000, 35, 4, 16, 32, 256, 8, 256 * 8, 0,
                                  16, 35 * 4, None, None)
    assert rc == 1 and b"branches" in h.vqgnn_last_error()
    # the same call with nb = 32 passes validation (not launched: n == B)
    rc = h.vqgnn_gather_codewords(16, 100, 100, 16, 35, 1000, 32, 4, 16, 32, 256, 8, 256 * 8, 0,
                                  16, 32 * 4, None, None)
    assert rc == 0
    # codebook-source SpMM: F / D = 32 code columns against 16 branches
    rc = h.vqgnn_spmm_task_cb(16, 100, 1000, 50, 16, 128, 128, 16, 32, 1000, 16, 8, 256 * 8, 16,
                              256, 4, 16, 128, 16, 16, 64, 0, 0, 16, None)
    assert rc == 1 and b"branches" in h.vqgnn_last_error()
    assert h.vqgnn_spmm_task_cb_supported(100, 50, 128, 128, 128, 1000, 32, 16, 256, 4) == 0
    assert h.vqgnn_spmm_task_cb_supported(100, 50, 128, 128, 128, 1000, 32, 32, 256, 4) == 1
    # the kernel's other limits, mirrored by the query
    assert h.vqgnn_spmm_task_cb_supported(100, 50, 128, 128, 128, 1000, 32, 32, 1281, 4) == 0
    assert h.vqgnn_spmm_task_cb_supported(100, 50, 128, 128, 128, 1000, 32, 32, 1024, 4) == 1
    assert h.vqgnn_spmm_task_cb_supported(100, 50, 96, 96, 96, 1000, 24, 24, 640, 4) == 1  # G = 8
    # M codeword rows + the zero row (codes >= M read it)
    assert h.vqgnn_spmm_task_cb_lds(256) == 257 * 512 and h.vqgnn_spmm_task_cb_lds(1024) == 1025 * 128
    assert h.vqgnn_spmm_task_cb_supported(1 << 24, 50, 128, 128, 128, 1000, 32, 32, 256, 4) == 0
    assert h.vqgnn_spmm_task_cb_supported(100, 5_000_000, 128, 128, 128, 1000, 32, 32, 256,
                                          4) == 0          # X past the 2 GiB near range
    assert h.vqgnn_spmm_task_cb_supported(100, 50, 128, 40, 128, 1000, 16, 16, 256, 4) == 0


def test_codebook_source_preferred_only_at_full_width():
    """The host layer takes the codebook source only where the whole 128-column
    tile's image fits (M <= 319 with its zero row); narrower tiles lose to the gather (DESIGN
    4.2d, profiles/r05_cb_m1024_probe.txt)."""
    from vq_gnn_amd import kernels
    assert kernels.codebook_source_preferred(256) and kernels.codebook_source_preferred(319)
    assert not kernels.codebook_source_preferred(320)
    assert not kernels.codebook_source_preferred(1024)


def test_ema_finalize_args_layout_matches_header(tmp_path):
    """The ctypes record (vq_gnn_amd._lib.EmaFinalizeArgs) has the C layout of
    include/vqgnn.h §4b's vqgnn_ema_finalize_args: every field's offset and
    the size, as gcc lays the header's struct out."""
    import ctypes
    import shutil
    import subprocess
    import pytest
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    names = [f[0] for f in L.EmaFinalizeArgs._fields_]
    src = tmp_path / "off.c"
    src.write_text(
        "#include <stdio.h>\n#include <stddef.h>\n#include \"vqgnn.h\"\n"
        "int main(void) {\n"
        + "".join(f'  printf("%zu\\n", offsetof(vqgnn_ema_finalize_args, {n}));\n' for n in names)
        + '  printf("%zu\\n", sizeof(vqgnn_ema_finalize_args));\n  return 0;\n}\n')
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True,
                                          text=True).stdout.split()]
    want = [getattr(L.EmaFinalizeArgs, n).offset for n in names] + \
        [ctypes.sizeof(L.EmaFinalizeArgs)]
    assert got == want


def test_fused_finalize_entry_checks_the_finalize_first():
    """vqgnn_spmm_task_cb_fin rejects a bad finalize record before any
    launch (dummy device addresses are never dereferenced)."""
    import ctypes
    h = L.lib()
    fin = L.EmaFinalizeArgs(ema_parts=16, nparts=1, zero_after=1, stat_count=100, nb=32, M=256,
                            D=4, W=6, ldw=8, decay=0.99, laplace=1, grad_scale=1.0,
                            epsilon=1e-5, cluster_size=16, cs_bstride=256, ema_w=16,
                            embedding=16, embedding_output=16, emb_bstride=2048, rm_f=16,
                            rv_f=16, rm_g=16, rv_g=16, bad_init=16)
    args = (16, 100, 1000, 50, 16, 128, 128, 16, 32, 1000, 16, 8, 2048, 32, 256, 4, 16, 128,
            16, 16, 64, 0, 0, 16)
    rc = h.vqgnn_spmm_task_cb_fin(*args, ctypes.byref(fin), None)
    assert rc == 1 and b"W must be D or 2D" in h.vqgnn_last_error()
    fin.W, fin.stat_count = 8, 0
    rc = h.vqgnn_spmm_task_cb_fin(*args, ctypes.byref(fin), None)
    assert rc == 1 and b"stat_count" in h.vqgnn_last_error()


def test_split_walk_and_fixup_check_like_the_one_call_entry():
    """vqgnn_spmm_task_cb_walk / _fixup (the walk beside the VQ update, its
    fix-up after both) run the one-call entry's checks before any launch:
    the branch bound, the tile limits, and (fix-up) the finalize record."""
    import ctypes
    h = L.lib()
    # F / D = 32 code columns against 16 branches: both halves refuse
    bad = (16, 100, 1000, 50, 16, 128, 128, 16, 32, 1000, 16, 8, 256 * 8, 16, 256, 4, 16, 128,
           16, 16, 64, 0, 0, 16)
    assert h.vqgnn_spmm_task_cb_walk(*bad, None) == 1
    assert b"branches" in h.vqgnn_last_error()
    assert h.vqgnn_spmm_task_cb_fixup(*bad, None, None) == 1
    assert b"branches" in h.vqgnn_last_error()
    # M past the widest image
    big = bad[:13] + (32, 1281) + bad[15:]
    assert h.vqgnn_spmm_task_cb_walk(*big, None) == 1 and b"image" in h.vqgnn_last_error()
    # the fix-up checks the finalize record first, as vqgnn_spmm_task_cb_fin
    fin = L.EmaFinalizeArgs(ema_parts=16, nparts=1, zero_after=1, stat_count=100, nb=32, M=256,
                            D=4, W=6, ldw=8, decay=0.99, laplace=1, grad_scale=1.0,
                            epsilon=1e-5, cluster_size=16, cs_bstride=256, ema_w=16,
                            embedding=16, embedding_output=16, emb_bstride=2048, rm_f=16,
                            rv_f=16, rm_g=16, rv_g=16, bad_init=16)
    good = bad[:13] + (32,) + bad[14:]
    assert h.vqgnn_spmm_task_cb_fixup(*good, ctypes.byref(fin), None) == 1
    assert b"W must be D or 2D" in h.vqgnn_last_error()


def test_default_library_reads_no_measurement_knobs():
    """The shipped library never reads the measurement knobs that cut work
    short or drop stores (VQGNN_TASK_DBG, VQGNN_ASSIGN_MSWEEP, the schedule
    and chunk knobs): they exist only in -DVQGNN_EXPERIMENTS builds
    (scripts/build_variant.sh).  The environment names it can read are the
    three alternative-implementation switches, whose results the suite checks
    equal to the default path's."""
    data = open(L._DEFAULT_LIB, "rb").read()
    names = set(m.decode() for m in re.findall(rb"VQGNN_[A-Z0-9_]+", data))
    assert names <= {"VQGNN_ASSIGN_EXACT", "VQGNN_EMA_GLOBAL", "VQGNN_SPMM_FAR"}, names
    for knob in (b"VQGNN_TASK_DBG", b"VQGNN_ASSIGN_MSWEEP", b"VQGNN_TASK_U", b"VQGNN_ASG_CHUNK"):
        assert knob not in data


def test_bn_fold_refuses_chunked_codebooks():
    """the BatchNorm fold is not offered for a codebook the assign
    stages in chunks (chunk-outer passes, ppi's M = 4,096), a combination no
    parity test pins; the single-chunk arxiv shape keeps it (host query)."""
    h = L.lib()
    assert h.vqgnn_vq_assign_bn_supported(30_000, 13, 4, 4096, 8) == 0
    assert h.vqgnn_vq_assign_bn_supported(84_670, 32, 4, 256, 8) == 1


def test_codebook_source_query_agrees_with_the_entry(monkeypatch):
    """the supported query refuses what the entry would refuse --
    VQGNN_SPMM_FAR (the entry needs the near path) -- and codebook_source_ok
    checks the codeword rows' layout the entry checks."""
    import torch
    from vq_gnn_amd import kernels
    h = L.lib()
    args = (100, 50, 128, 128, 128, 1000, 32, 32, 256, 4)
    assert h.vqgnn_spmm_task_cb_supported(*args) == 1
    monkeypatch.setenv("VQGNN_SPMM_FAR", "1")
    assert h.vqgnn_spmm_task_cb_supported(*args) == 0
    monkeypatch.delenv("VQGNN_SPMM_FAR")
    X = torch.zeros(50, 128)
    good = torch.zeros(32, 256, 8)
    assert kernels.codebook_source_ok(X, 128, 256, 4, n_rows=100, emb_out=good)
    odd = torch.zeros(32, 256, 10)[:, :, :6]          # ldw = 10: not a multiple of 4
    assert not kernels.codebook_source_ok(X, 128, 256, 4, n_rows=100, emb_out=odd)


def test_assign_kernels_have_no_packed_fp32():
    """The assign kernels are built without SLP vectorization (csrc/Makefile):
    no packed FP32 instruction in any vq_filter_kernel / vq_assign_kernel
    instance, so the resolve's exact candidate chains are v_fma_f32 chains in
    every instance (round 5's nondeterministic variant ran them packed;
    DESIGN.md 4.1).  Reads the gfx950 code object of the built library."""
    import subprocess
    import tempfile
    import pytest
    llvm = "/opt/rocm/lib/llvm/bin"
    obj = os.path.join(ROOT, "vq-gnn_amd", "lib", "obj", "vq_kernels.o")
    if not (os.path.exists(obj) and os.path.exists(os.path.join(llvm, "llvm-objdump"))):
        pytest.skip("needs the built object and the ROCm LLVM tools")
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.run([f"{llvm}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj,
                        os.path.join(d, "host.o")], check=True)
        subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                        f"--output={dev}"], check=True)
        asm = subprocess.run([f"{llvm}/llvm-objdump", "-d", dev], check=True,
                             capture_output=True, text=True).stdout
    funcs = re.split(r"\n(?=[0-9a-f]+ <)", asm)
    assign = [f for f in funcs if "vq_filter_kernel" in f.split("\n", 1)[0] or
              "vq_assign_kernel" in f.split("\n", 1)[0]]
    assert len(assign) >= 18
    for f in assign:
        packed = re.findall(r"\bv_pk_(?:fma|mul|add)_f32\b", f)
        assert not packed, (f.split("\n", 1)[0][:80], len(packed))
