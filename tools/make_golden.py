"""Generates the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container (it reads /root/reference; nothing on the GPU box
needs it).  Run with PYTHONDONTWRITEBYTECODE=1 (it also sets
sys.dont_write_bytecode) so nothing is written under /root/reference.

Sources of expected outputs:
  * C++  -- the reference's own "C++ Codes/modules/ACA_SKS.cpp", compiled by
            oracle/build.sh into oracle/_ref/libsks_ref.so (normalised H, f32 & f64).
  * PyTorch -- the reference's own statements of TensorACA_rect and ACA_vanilla
            ("PyTorch Codes/Modules_Runtime_Test.py:294-302, :330-383") and of its
            input generators (:9-37), executed verbatim on CPU torch.  The module is
            not imported (its top level imports torchgeometry, absent here): the
            script parses the file and executes those functions' own statements,
            dropping only the timing lines of the loop bodies (torch.cuda.synchronize,
            perf_counter, time_list).
  * Matlab -- veri_4Pts.m's camera model restated in numpy (no Octave here): the
            known-answer H_real for the KAT quad (veri_4Pts.m:9-53) and rectangle
            (:82-93).
Inputs include the reference's own correspondence file
("C++ Codes/Runtime Test/CPU_Runtime Test/orig_pts_wall.txt").

Every fixture stores inputs and expected outputs as raw float32/float64 arrays.
"""
from __future__ import annotations

import ast
import os
import sys

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("SKS_REFERENCE_ROOT", "/root/reference")
PY_REF = os.path.join(REF, "PyTorch Codes", "Modules_Runtime_Test.py")
WALL = os.path.join(REF, "C++ Codes", "Runtime Test", "CPU_Runtime Test", "orig_pts_wall.txt")
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle import RefOracle  # noqa: E402


# ------------------------------------------------------------ python reference
def _ref_functions():
    tree = ast.parse(open(PY_REF).read(), PY_REF)
    return {n.name: n for n in tree.body if isinstance(n, ast.FunctionDef)}


_TIMING_TOKENS = ("torch.cuda.synchronize", "perf_counter", "time_list")


def _loop_body(fn: ast.FunctionDef, src_text: str) -> ast.Module:
    """The statements of the function's timing loop, minus the timing statements."""
    loops = [n for n in fn.body if isinstance(n, ast.For)]
    assert len(loops) == 1, fn.name
    keep = [s for s in loops[0].body
            if not any(tok in ast.get_source_segment(src_text, s) for tok in _TIMING_TOKENS)]
    return ast.Module(body=keep, type_ignores=[])


def run_ref_statements(name: str, **env):
    text = open(PY_REF).read()
    fns = _ref_functions()
    mod = _loop_body(fns[name], text)
    ns = {"torch": torch, **env}
    exec(compile(mod, f"{PY_REF}:{name}", "exec"), ns)
    return ns


def ref_generators():
    fns = _ref_functions()
    mod = ast.Module(body=[fns["getInput"], fns["getTar"], fns["adjust"]], type_ignores=[])
    ns = {"torch": torch}
    exec(compile(mod, f"{PY_REF}:generators", "exec"), ns)
    return ns


# ----------------------------------------------------------------- data helpers
def read_wall():
    """orig_pts_wall.txt parsed as the reference parses it: sscanf("%f") = C strtof, one
    rounding to binary32 (not float() then float32, which rounds twice)."""
    import ctypes
    import ctypes.util
    strtof = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6").strtof
    strtof.restype, strtof.argtypes = ctypes.c_float, [ctypes.c_char_p, ctypes.c_void_p]
    with open(WALL) as f:
        count = int(f.readline().split()[0])
        rows = [[strtof(v.encode(), None) for v in f.readline().split()[:4]] for _ in range(count)]
    a = np.asarray(rows, dtype=np.float32)
    return a[:, 0:2], a[:, 2:4]


def wall_problems(n, seed):
    ps, pt = read_wall()
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, ps.shape[0], size=(n, 4))
    return ps[idx].reshape(n, 8), pt[idx].reshape(n, 8), idx.astype(np.uint32)


def edge_problems():
    """Degenerate and extreme quads (duplicates, collinear triples, zero/huge/
    negative/subnormal coordinates, NaN/Inf inputs, integer grids)."""
    rng = np.random.default_rng(7)
    base_s = np.array([0, 0, 200, 0, 50, 139, 181, 93], np.float32)
    base_t = np.array([10, 12, 220, 5, 40, 160, 190, 110], np.float32)
    cases = []

    def add(s, t):
        cases.append((np.asarray(s, np.float32), np.asarray(t, np.float32)))

    add(base_s, base_t)
    add(base_s, base_s)                                     # identity
    add(np.zeros(8), np.zeros(8))                           # everything coincident
    s = base_s.copy(); s[2:4] = s[0:2]; add(s, base_t)      # M == N
    s = base_s.copy(); s[6:8] = s[4:6]; add(s, base_t)      # P == Q
    t = base_t.copy(); t[4:6] = t[0:2]; add(base_s, t)      # target M == P
    add([0, 0, 1, 1, 2, 2, 3, 7], base_t)                   # collinear M, N, P
    add(base_s, [0, 0, 10, 0, 20, 0, 5, 9])                 # collinear target M, N, P
    add([0, 0, 1, 0, 0, 1, 1, 1], [0, 0, 1, 0, 0, 1, 1, 1])  # unit square
    add([0, 0, 1, 0, 0, 1, 1, 1], [0, 0, 2, 0, 0, 2, 2, 2])
    add(-base_s, base_t)                                    # negative coordinates
    add(base_s * 1e6, base_t * 1e6)                         # huge
    add(base_s * 1e18, base_t * 1e18)                       # overflow territory
    add(base_s * 1e-20, base_t * 1e-20)                     # underflow / subnormal
    add(base_s * np.float32(1e-39), base_t)                 # subnormal source
    s = base_s.copy(); s[3] = np.nan; add(s, base_t)        # NaN input
    t = base_t.copy(); t[0] = np.inf; add(base_s, t)        # Inf input
    add([0, 0, 0, 0, 0, 0, 0, 0], base_t)                   # zero-area source
    for k in range(16):                                     # integer grids
        g = rng.integers(-64, 64, size=8).astype(np.float32)
        h = rng.integers(-64, 64, size=8).astype(np.float32)
        add(g, h)
    for k in range(16):                                     # tiny perturbations of a square
        sq = np.array([0, 0, 1, 0, 0, 1, 1, 1], np.float32) * 100
        add(sq + rng.normal(0, 1e-3, 8).astype(np.float32), sq)
    for k in range(14):                                     # wide dynamic range
        add(rng.uniform(-1, 1, 8).astype(np.float32) * np.float32(10.0 ** rng.integers(-8, 8)),
            rng.uniform(-1, 1, 8).astype(np.float32) * np.float32(10.0 ** rng.integers(-8, 8)))
    src = np.stack([c[0] for c in cases])
    tar = np.stack([c[1] for c in cases])
    return src, tar


# --------------------------------------------------------------- Matlab KAT
def veri_4pts():
    """Camera model of veri_4Pts.m:28-53 (K, R = Rx*Ry*Rz, T) restated in numpy."""
    fu = fv = 900.0
    u0, v0 = 500.0, 400.0
    K = np.array([[fu, 0, u0], [0, fv, v0], [0, 0, 1.0]])
    rx = -np.pi / 8 * np.sqrt(5)
    ry = -np.pi / 8 * np.sqrt(5)
    rz = -np.pi / 16 * np.sqrt(5)
    Rx = np.array([[1, 0, 0], [0, np.cos(rx), -np.sin(rx)], [0, np.sin(rx), np.cos(rx)]])
    Ry = np.array([[np.cos(ry), 0, np.sin(ry)], [0, 1, 0], [-np.sin(ry), 0, np.cos(ry)]])
    Rz = np.array([[np.cos(rz), -np.sin(rz), 0], [np.sin(rz), np.cos(rz), 0], [0, 0, 1]])
    R = Rx @ Ry @ Rz
    T = np.array([-10.5, -12.5, 525.0])
    H_real = K @ np.column_stack([R[:, 0], R[:, 1], T])
    src = np.array([[0, 0], [200, 0], [50, 139], [181, 93]], dtype=np.float64)   # :9-12

    def project(pts):
        ph = H_real @ np.vstack([pts.T, np.ones(len(pts))])
        return (ph[:2] / ph[2]).T

    tar = project(src)
    # rectangle case (:82-93): width 50, height 40, M = (36, 81), order M N P Q
    w, h, mx, my = 50.0, 40.0, 36.0, 81.0
    rect = np.array([[mx, my], [mx + w, my], [mx, my + h], [mx + w, my + h]])
    rect_tar = project(rect)
    return H_real, src, tar, rect, rect_tar, (w, h, mx, my)


def main():
    os.makedirs(OUT, exist_ok=True)
    ref = RefOracle()
    manifest = []

    # 1. uniform random quads (f32 + f64) -- C++ reference, normalised
    rng = np.random.default_rng(2025)
    n = 1024
    s32 = rng.uniform(0, 1024, (n, 8)).astype(np.float32)
    t32 = rng.uniform(0, 1024, (n, 8)).astype(np.float32)
    s64 = rng.uniform(-512, 512, (n, 8))
    t64 = rng.uniform(-512, 512, (n, 8))
    np.savez(os.path.join(OUT, "cpp_uniform.npz"), src_f32=s32, tar_f32=t32,
             aca_f32=ref.solve("aca", s32, t32), sks_f32=ref.solve("sks", s32, t32),
             ge_f32=ref.solve("ge", s32, t32),
             src_f64=s64, tar_f64=t64, aca_f64=ref.solve("aca", s64, t64),
             sks_f64=ref.solve("sks", s64, t64))
    manifest.append("cpp_uniform.npz: 1024 U[0,1024) f32 + 1024 U[-512,512) f64 quads; "
                    "sks::runKernel_{ACA,SKS}[_double] outputs (reference C++)")

    # 2. the reference's own correspondence file, random 4-subsets
    ws, wt, widx = wall_problems(1024, 11)
    ps, pt = read_wall()
    np.savez(os.path.join(OUT, "cpp_wall.npz"), src=ws, tar=wt, idx=widx, pool_src=ps,
             pool_tar=pt, aca=ref.solve("aca", ws, wt), sks=ref.solve("sks", ws, wt),
             ge=ref.solve("ge", ws, wt))
    manifest.append("cpp_wall.npz: 1024 4-subsets of orig_pts_wall.txt (reference data file), "
                    "pool + indices kept for the fused sampler; reference C++ outputs")
    with open(os.path.join(OUT, "orig_pts_wall_restated.txt"), "w") as f:
        f.write(f"{ps.shape[0]}\n")
        for a, b in zip(ps, pt):
            f.write(" ".join(np.format_float_positional(v, unique=True)
                             for v in (a[0], a[1], b[0], b[1])) + "\n")
    manifest.append("orig_pts_wall_restated.txt: the pool of cpp_wall.npz written back in the "
                    "reference's point-file format (count line, then x1 y1 x2 y2; shortest "
                    "round-trip decimals) -- input for examples/runtime_test.cpp")

    # 3. edge cases, f32 and f64
    es, et = edge_problems()
    np.savez(os.path.join(OUT, "cpp_edge.npz"), src=es, tar=et,
             aca=ref.solve("aca", es, et), sks=ref.solve("sks", es, et),
             ge=ref.solve("ge", es, et),
             src_f64=es.astype(np.float64), tar_f64=et.astype(np.float64),
             aca_f64=ref.solve("aca", es.astype(np.float64), et.astype(np.float64)),
             sks_f64=ref.solve("sks", es.astype(np.float64), et.astype(np.float64)))
    manifest.append(f"cpp_edge.npz: {len(es)} degenerate/extreme quads (duplicates, collinear, "
                    "zero/huge/subnormal/NaN/Inf, integer grids); reference C++ outputs")

    # 4. Matlab KAT
    H_real, ks, kt, rect, rect_tar, (w, h, mx, my) = veri_4pts()
    ks32, kt32 = ks.reshape(1, 8).astype(np.float32), kt.reshape(1, 8).astype(np.float32)
    np.savez(os.path.join(OUT, "kat_veri4pts.npz"), H_real=H_real,
             H_real_norm=H_real / H_real[2, 2], src=ks.reshape(1, 8), tar=kt.reshape(1, 8),
             src_f32=ks32, tar_f32=kt32, aca_f32=ref.solve("aca", ks32, kt32),
             sks_f32=ref.solve("sks", ks32, kt32),
             aca_f64=ref.solve("aca", ks.reshape(1, 8), kt.reshape(1, 8)),
             sks_f64=ref.solve("sks", ks.reshape(1, 8), kt.reshape(1, 8)),
             rect_src=rect, rect_tar=rect_tar, rect_whm=np.array([w, h, mx, my]))
    manifest.append("kat_veri4pts.npz: veri_4Pts.m camera-model KAT (H_real, projected quad and "
                    "rectangle) + reference C++ outputs on it")

    # 5. PyTorch reference: TensorACA_rect and ACA_vanilla statements, CPU torch
    gen = ref_generators()
    torch.manual_seed(0)
    B = 256
    src, tar, src_h, tar_h, scale, div = gen["adjust"]("cpu", B)
    ns = run_ref_statements("TensorACA_rect", bs=B, src=src_h, tar=tar_h, scale=scale, div=div)
    H_rect_int = ns["H"].numpy().copy()
    ns = run_ref_statements("ACA_vanilla", bs=B, src=src, tar=tar)
    H_van_int = ns["H"].numpy().copy()
    # non-integer inputs (exercises every rounding of the formulation)
    g = torch.Generator().manual_seed(5)
    src2 = torch.rand((B, 4, 2), generator=g) * 128 + torch.tensor([[0, 0], [128, 0], [0, 128],
                                                                    [128, 128.0]])
    tar2 = src2 + torch.rand((B, 4, 2), generator=g) * 32
    ones = torch.ones((B, 1, 4))
    src2_h = torch.cat((src2.transpose(1, 2), ones), dim=1)
    tar2_h = torch.cat((tar2.transpose(1, 2), ones), dim=1)
    sc2 = torch.tensor([128.0])
    dv2 = torch.tensor([1.0])
    # rectangle with a non-square aspect, like veri_4Pts's 50x40 (div = 1.25)
    sc3 = torch.tensor([50.0])
    dv3 = torch.tensor([1.25])
    H_rect_f = run_ref_statements("TensorACA_rect", bs=B, src=src2_h, tar=tar2_h, scale=sc2,
                                  div=dv2)["H"].numpy().copy()
    H_rect_f3 = run_ref_statements("TensorACA_rect", bs=B, src=src2_h, tar=tar2_h, scale=sc3,
                                   div=dv3)["H"].numpy().copy()
    H_van_f = run_ref_statements("ACA_vanilla", bs=B, src=src2, tar=tar2)["H"].numpy().copy()
    np.savez(os.path.join(OUT, "torch_tensor_aca.npz"),
             int_src=src.numpy(), int_tar=tar.numpy(), int_src_h=src_h.numpy(),
             int_tar_h=tar_h.numpy(), int_scale=scale.numpy(), int_div=div.numpy(),
             int_rect=H_rect_int, int_vanilla=H_van_int,
             f_src=src2.numpy(), f_tar=tar2.numpy(), f_src_h=src2_h.numpy(),
             f_tar_h=tar2_h.numpy(), f_rect=H_rect_f, f_rect_div125=H_rect_f3,
             f_vanilla=H_van_f)
    manifest.append("torch_tensor_aca.npz: TensorACA_rect / ACA_vanilla statements of the "
                    "reference executed on CPU torch %s (ATen CPU capability %s): 256 "
                    "adjust() batches (seed 0) + 256 non-integer batches (scale 128/div 1 and "
                    "scale 50/div 1.25)" % (torch.__version__,
                                            torch.backends.cpu.get_cpu_capability()))

    manifest.append(torch_special())

    # 6. the reference input generator itself (seed 0, B=8)
    torch.manual_seed(0)
    out = gen["adjust"]("cpu", 8)
    np.savez(os.path.join(OUT, "torch_generator.npz"),
             **{k: v.numpy() for k, v in zip(["src", "tar", "src_h", "tar_h", "scale", "div"],
                                            out)})
    manifest.append("torch_generator.npz: reference adjust('cpu', 8) after torch.manual_seed(0)")

    with open(os.path.join(OUT, "MANIFEST.txt"), "w") as f:
        f.write("Golden fixtures, generated by tools/make_golden.py from the reference itself.\n")
        f.write("torch %s, numpy %s\n\n" % (torch.__version__, np.__version__))
        for m in manifest:
            f.write("- " + m + "\n")
    print("\n".join(manifest))


def torch_special() -> str:
    """TensorACA_rect / ACA_vanilla statements of the reference on special values, CPU torch:
    signed zeros, +-Inf, NaN, subnormals, near-overflow and ties (4096 problems each), the
    all-(-0) cross-product case (torch.sum's +0 accumulator decides its sign), and quads over
    24 decades of scale.  Writes tests/golden/torch_special.npz; returns its manifest line."""
    rng = np.random.default_rng(20261016)
    vals = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 3.0, 1024.0, np.inf, -np.inf, np.nan,
                     1e-45, -1.2e-40, 3e38, -3e38], np.float32)
    w = np.array([8, 6, 8, 6, 6, 4, 4, 4, 1, 1, 1, 1, 1, 1, 1], np.float64)
    B = 4096
    rect_src = rng.choice(vals, size=(B, 3, 4), p=w / w.sum()).astype(np.float32)
    rect_tar = rng.choice(vals, size=(B, 3, 4), p=w / w.sum()).astype(np.float32)
    # problem 0: every cross term -0 (underflowing products of tiny differences)
    rect_src[0] = 2.0
    rect_tar[0] = [[1.4e-45, -0.0, 0.0, 0.0], [-1.2e-40, 0.0, -0.0, 0.0], [-0.0, 1024.0, -0.0, 0.0]]
    scaled = lambda: (rng.uniform(-1, 1, (B, 4, 2)) *  # noqa: E731
                      10.0 ** rng.integers(-12, 13, (B, 1, 1))).astype(np.float32)
    van_src, van_tar = scaled(), scaled()
    k = B // 4  # a quarter of the quads with special coordinates mixed in
    van_src[:k] = rng.choice(vals, size=(k, 4, 2), p=w / w.sum())
    out = {"rect_src": rect_src, "rect_tar": rect_tar, "van_src": van_src, "van_tar": van_tar}
    for tag, sc, dv in (("128_1", 128.0, 1.0), ("50_125", 50.0, 1.25), ("inf_05", np.inf, 0.5)):
        out[f"rect_{tag}"] = run_ref_statements(
            "TensorACA_rect", bs=B, src=torch.from_numpy(rect_src), tar=torch.from_numpy(rect_tar),
            scale=torch.tensor([sc], dtype=torch.float32),
            div=torch.tensor([dv], dtype=torch.float32))["H"].numpy().copy()
    out["vanilla"] = run_ref_statements("ACA_vanilla", bs=B, src=torch.from_numpy(van_src),
                                        tar=torch.from_numpy(van_tar))["H"].numpy().copy()
    np.savez_compressed(os.path.join(OUT, "torch_special.npz"), **out)
    return ("torch_special.npz: TensorACA_rect (scale/div 128/1, 50/1.25, inf/0.5) and ACA_vanilla "
            "statements of the reference on CPU torch %s (ATen CPU capability %s) over 4096 "
            "special-value problems each (signed zeros, +-Inf, NaN, subnormals, near-overflow; "
            "problem 0 of rect: all three cross terms -0) and 24 decades of scale" %
            (torch.__version__, torch.backends.cpu.get_cpu_capability()))


def torch_aca_f64() -> str:
    """ACA_vanilla's own statements (Modules_Runtime_Test.py:322-382) executed on float64 CPU
    tensors -- binary64 ACA without normalisation, the contract of the reference GPU kernel
    cal_Homo_ACA (GPU_Runtime Test.cu:81-151).  The statements allocate H with torch.ones
    (default dtype), so torch's default dtype is float64 while they run; every other tensor
    follows the float64 inputs.  Inputs: uniform quads, 4-subsets of the reference's point
    file (Point2f read as the harness reads it, widened to Point2d as .cu:1414-1416 does) and
    the edge set.  Writes tests/golden/torch_aca_f64.npz; returns its manifest line."""
    rng = np.random.default_rng(64)
    n = 1024
    uni_s = rng.uniform(-512, 512, (n, 4, 2))
    uni_t = rng.uniform(-512, 512, (n, 4, 2))
    ws, wt, widx = wall_problems(n, 64)
    es, et = edge_problems()
    out = {"wall_idx": widx}
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        for tag, src, tar in (("uniform", uni_s, uni_t),
                              ("wall", ws.astype(np.float64).reshape(n, 4, 2),
                               wt.astype(np.float64).reshape(n, 4, 2)),
                              ("edge", es.astype(np.float64).reshape(-1, 4, 2),
                               et.astype(np.float64).reshape(-1, 4, 2))):
            H = run_ref_statements("ACA_vanilla", bs=src.shape[0], src=torch.from_numpy(src),
                                   tar=torch.from_numpy(tar))["H"]
            assert H.dtype == torch.float64
            out[f"{tag}_src"], out[f"{tag}_tar"] = src, tar
            out[f"{tag}_H"] = H.numpy().copy()
    finally:
        torch.set_default_dtype(prev)
    np.savez_compressed(os.path.join(OUT, "torch_aca_f64.npz"), **out)
    return ("torch_aca_f64.npz: ACA_vanilla statements of the reference on float64 CPU torch %s "
            "(unnormalised binary64 ACA, the cal_Homo_ACA contract): 1024 uniform quads, 1024 "
            "4-subsets of orig_pts_wall.txt, %d edge cases" % (torch.__version__, len(es)))


BCAST_SHAPES = ["()", "(1,)", "(1,1,1)", "(1,1,1,1)", "(B,1,1)", "(1,B,1,1)", "(3,1)", "(1,3,1)",
                "(B,3,1)", "(B,)", "(B,1)", "(3,)", "(2,)", "(B,3)", "(B,3,2)", "(2,B,3,1)",
                "(2,1,1,1)"]


def torch_bcast() -> str:
    """TensorACA_rect's own statements (Modules_Runtime_Test.py:294-302) with scale / div of
    every shape in BCAST_SHAPES (B = 64), on CPU torch: whether the composition accepts the
    shape (its broadcasting and the (B,3,1) column assignment decide), H where it does, and
    the gradients ATen autograd gives through those statements (dL/dtar, dL/dscale, dL/ddiv
    for L = sum(H * gH)).  scale and div get the same shape in each case, plus two mixed
    cases.  Writes tests/golden/torch_rect_bcast.npz; returns its manifest line."""
    B = 64
    g = torch.Generator().manual_seed(77)
    src = torch.rand((B, 4, 2), generator=g) * 128 + torch.tensor([[0, 0], [128, 0], [0, 128],
                                                                   [128, 128.0]])
    tar = src + torch.rand((B, 4, 2), generator=g) * 32
    ones = torch.ones((B, 1, 4))
    src_h = torch.cat((src.transpose(1, 2), ones), dim=1)
    tar_h = torch.cat((tar.transpose(1, 2), ones), dim=1)
    gH = torch.randn((B, 3, 3), generator=g)
    out = {"src_h": src_h.numpy(), "tar_h": tar_h.numpy(), "gH": gH.numpy()}
    cases = [(sh, sh) for sh in BCAST_SHAPES] + [("(1,)", "(B,1,1)"), ("(3,1)", "(B,3,1)")]
    names, accepted = [], []
    for k, (ss, ds) in enumerate(cases):
        shp = lambda t: tuple(eval(t, {"B": B}))  # noqa: E731
        scale = (torch.rand(shp(ss), generator=g) * 64 + 64).float()
        div = (torch.rand(shp(ds), generator=g) + 0.5).float()
        tr = tar_h.clone().requires_grad_(True)
        sc = scale.clone().requires_grad_(True)
        dv = div.clone().requires_grad_(True)
        try:
            H = run_ref_statements("TensorACA_rect", bs=B, src=src_h, tar=tr, scale=sc,
                                   div=dv)["H"]
            ok = True
        except RuntimeError:
            ok = False
        names.append(f"{ss}|{ds}")
        accepted.append(ok)
        out[f"c{k}_scale"], out[f"c{k}_div"] = scale.numpy(), div.numpy()
        if ok:
            (H * gH).sum().backward()
            out[f"c{k}_H"] = H.detach().numpy().copy()
            out[f"c{k}_gtar"] = tr.grad.numpy().copy()
            out[f"c{k}_gscale"] = sc.grad.numpy().copy()
            out[f"c{k}_gdiv"] = dv.grad.numpy().copy()
    out["cases"] = np.array(names)
    out["accepted"] = np.array(accepted)
    np.savez_compressed(os.path.join(OUT, "torch_rect_bcast.npz"), **out)
    return ("torch_rect_bcast.npz: TensorACA_rect statements of the reference on CPU torch %s "
            "(ATen CPU capability %s), B = 64, scale/div of %d shapes (accepted or refused by "
            "the composition itself), H and the ATen autograd gradients of sum(H * gH)"
            % (torch.__version__, torch.backends.cpu.get_cpu_capability(), len(cases)))


def torch_rect_grad() -> str:
    """The gradients ATen autograd gives through TensorACA_rect's own statements
    (Modules_Runtime_Test.py:294-302) on CPU torch: dL/dtar, dL/dscale, dL/ddiv for
    H.backward(gH), src held constant -- with src requiring grad the statements fail in
    backward (H is written in place after column 2 has read columns 0 and 1), which is
    recorded too.  Cases: the reference's own adjust() batches (seed 0) with integer gH full
    of signed zeros and identity problems (all cross terms 0); fractional quads; special
    values; random bit patterns; per-problem (B,1,1) and per-(problem, row) (B,3,1)
    scale / div.  Writes tests/golden/torch_rect_grad.npz; returns its manifest line."""
    gen = ref_generators()
    rng = np.random.default_rng(4242)
    out = {}
    vals = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 1024.0, np.inf, -np.inf, np.nan, 1e-45,
                     -1.2e-40, 3e38], np.float32)

    def frac(B):
        g = torch.Generator().manual_seed(B)
        s = torch.rand((B, 4, 2), generator=g) * 128 + torch.tensor([[0, 0], [128, 0], [0, 128],
                                                                     [128, 128.0]])
        t = s + torch.rand((B, 4, 2), generator=g) * 32
        ones = torch.ones((B, 1, 4))
        return (torch.cat((s.transpose(1, 2), ones), dim=1).numpy(),
                torch.cat((t.transpose(1, 2), ones), dim=1).numpy())

    cases = []
    torch.manual_seed(0)
    B = 2048
    _, _, s_int, t_int, sc_int, dv_int = gen["adjust"]("cpu", B)
    s_int, t_int = s_int.numpy().copy(), t_int.numpy().copy()
    t_int[: B // 16, 0:2, :] = s_int[: B // 16, 0:2, :]  # identity problems
    g_int = rng.integers(-3, 4, (B, 3, 3)).astype(np.float32)
    g_int[rng.random((B, 3, 3)) < 0.3] = -0.0
    g_int[B // 16: B // 8] = -0.0
    cases.append(("int", s_int, t_int, g_int, sc_int.numpy(), dv_int.numpy()))
    s_f, t_f = frac(B)
    cases.append(("frac", s_f, t_f, rng.standard_normal((B, 3, 3)).astype(np.float32),
                  np.array([50.0], np.float32), np.array([1.25], np.float32)))
    Bs = 1024
    pick = lambda *shape: rng.choice(vals, size=shape).astype(np.float32)  # noqa: E731
    for tag, sc, dv in (("special", 50.0, 1.25), ("special_inf", np.inf, 0.5)):
        cases.append((tag, pick(Bs, 3, 4), pick(Bs, 3, 4), pick(Bs, 3, 3),
                      np.array([sc], np.float32), np.array([dv], np.float32)))
    bits = lambda *shape: rng.integers(0, 2**32 - 1, size=shape, dtype=np.uint32,  # noqa: E731
                                       endpoint=True).view(np.float32)
    cases.append(("bits", bits(Bs, 3, 4), bits(Bs, 3, 4), bits(Bs, 3, 3),
                  np.array([50.0], np.float32), np.array([1.25], np.float32)))
    s_p, t_p = frac(Bs)
    g_p = rng.standard_normal((Bs, 3, 3)).astype(np.float32)
    cases.append(("per_problem", s_p, t_p, g_p,
                  (rng.random((Bs, 1, 1)) * 64 + 64).astype(np.float32),
                  (rng.random((Bs, 1, 1)) + 0.5).astype(np.float32)))
    cases.append(("per_row", s_p, t_p, g_p, (rng.random((Bs, 3, 1)) * 64 + 64).astype(np.float32),
                  (rng.random((Bs, 3, 1)) + 0.5).astype(np.float32)))
    names = []
    for tag, src, tar, gH, scale, div in cases:
        tr = torch.from_numpy(tar.copy()).requires_grad_(True)
        sc = torch.from_numpy(scale.copy()).requires_grad_(True)
        dv = torch.from_numpy(div.copy()).requires_grad_(True)
        H = run_ref_statements("TensorACA_rect", bs=tar.shape[0], src=torch.from_numpy(src),
                               tar=tr, scale=sc, div=dv)["H"]
        H.backward(torch.from_numpy(gH))
        names.append(tag)
        out.update({f"{tag}_src": src, f"{tag}_tar": tar, f"{tag}_gH": gH, f"{tag}_scale": scale,
                    f"{tag}_div": div, f"{tag}_gtar": tr.grad.numpy().copy(),
                    f"{tag}_gscale": sc.grad.numpy().copy(), f"{tag}_gdiv": dv.grad.numpy().copy()})
    # src requiring grad: the statements' backward refuses (in-place H)
    sr = torch.from_numpy(s_f.copy()).requires_grad_(True)
    H = run_ref_statements("TensorACA_rect", bs=B, src=sr, tar=torch.from_numpy(t_f),
                           scale=torch.tensor([50.0]), div=torch.tensor([1.25]))["H"]
    try:
        H.backward(torch.ones_like(H))
        refused = False
    except RuntimeError:
        refused = True
    out["src_grad_refused"] = np.array(refused)
    out["cases"] = np.array(names)
    np.savez_compressed(os.path.join(OUT, "torch_rect_grad.npz"), **out)
    return ("torch_rect_grad.npz: ATen autograd through the reference's TensorACA_rect statements "
            "on CPU torch %s (ATen CPU capability %s): dL/dtar, dL/dscale, dL/ddiv for "
            "H.backward(gH) on %s (src constant: with src requiring grad the statements' "
            "backward raises -- recorded: %s)" % (torch.__version__,
                                                   torch.backends.cpu.get_cpu_capability(),
                                                   ", ".join(names), refused))


RECT_GRAD_LARGE_B = (65536, 1048576)
RECT_GRAD_LARGE_THREADS = (1, 4, 8, 16)
RECT_GRAD_LARGE_SEED = 2026


def torch_rect_grad_large() -> str:
    """ATen autograd's batch-uniform scale / div gradients through TensorACA_rect's own
    statements (Modules_Runtime_Test.py:294-302) on CPU torch at B = 64 K (BASELINE configs[3])
    and 1 M -- sums of 3B float32 terms whose order depends on at::get_num_threads(), so each
    is recorded for several thread counts (torch.set_num_threads).  Inputs are regenerated
    from oracle.rect_grad_batch (fill_uniform counter streams), not stored; dL/dtar is kept
    as a SHA-256 of its bytes.  A (3,1) per-row scale / div case (column sums, independent of
    the thread count) rides along.  Writes tests/golden/torch_rect_grad_large.npz."""
    import hashlib
    from oracle import Oracle, rect_grad_batch
    o = Oracle()
    out = {"B": np.array(RECT_GRAD_LARGE_B), "threads": np.array(RECT_GRAD_LARGE_THREADS),
           "seed": np.array(RECT_GRAD_LARGE_SEED)}
    prev = torch.get_num_threads()
    try:
        for B in RECT_GRAD_LARGE_B:
            sh, th, gH = rect_grad_batch(o, B, RECT_GRAD_LARGE_SEED + B)
            cases = [("uniform", np.array([128.0], np.float32), np.array([1.0], np.float32), RECT_GRAD_LARGE_THREADS),
                     ("frac", np.array([50.0], np.float32), np.array([1.25], np.float32), RECT_GRAD_LARGE_THREADS),
                     ("per_row", o.fill_uniform(3, 7, 0, 64.0, 128.0).reshape(3, 1),
                      o.fill_uniform(3, 7, 3, 0.5, 1.5).reshape(3, 1), (1, 8))]
            for tag, scale, div, threads in cases:
                for T in threads:
                    torch.set_num_threads(T)
                    tr = torch.from_numpy(th.copy()).requires_grad_(True)
                    sc = torch.from_numpy(scale.copy()).requires_grad_(True)
                    dv = torch.from_numpy(div.copy()).requires_grad_(True)
                    H = run_ref_statements("TensorACA_rect", bs=B, src=torch.from_numpy(sh),
                                           tar=tr, scale=sc, div=dv)["H"]
                    H.backward(torch.from_numpy(gH))
                    key = f"B{B}_{tag}"
                    out[f"{key}_scale"], out[f"{key}_div"] = scale, div
                    out[f"{key}_T{T}_gscale"] = sc.grad.numpy().copy()
                    out[f"{key}_T{T}_gdiv"] = dv.grad.numpy().copy()
                    out[f"{key}_T{T}_gtar_sha256"] = np.array(
                        hashlib.sha256(np.ascontiguousarray(tr.grad.numpy()).tobytes()).hexdigest())
    finally:
        torch.set_num_threads(prev)
    np.savez_compressed(os.path.join(OUT, "torch_rect_grad_large.npz"), **out)
    return ("torch_rect_grad_large.npz: ATen autograd through the reference's TensorACA_rect "
            "statements on CPU torch %s (ATen CPU capability %s; sum kernel 8 lanes): dL/dscale, "
            "dL/ddiv (batch-uniform (1,), and (3,1) per row) and SHA-256 of dL/dtar at B = %s, "
            "for at::get_num_threads() in %s; inputs regenerated by oracle.rect_grad_batch"
            % (torch.__version__, torch.backends.cpu.get_cpu_capability(),
               ", ".join(map(str, RECT_GRAD_LARGE_B)), RECT_GRAD_LARGE_THREADS))


def torch_vanilla_grad() -> str:
    """The gradients ATen autograd gives through ACA_vanilla's own statements
    (Modules_Runtime_Test.py:322-382) on CPU torch: dL/dsrc, dL/dtar for H.backward(gH).
    binary32: uniform quads, the reference's adjust() batches (seed 0) with integer gH full of
    signed zeros, 4-subsets of the reference's point file, the edge set, special values and
    random bit patterns; binary64 (the statements run with float64 as the default dtype, as
    torch_aca_f64 does): uniform quads, point-file subsets, the edge set.  Writes
    tests/golden/torch_vanilla_grad.npz; returns its manifest line."""
    gen = ref_generators()
    rng = np.random.default_rng(3141)
    vals = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 1024.0, np.inf, -np.inf, np.nan, 1e-45,
                     -1.2e-40, 3e38], np.float32)
    n = 512
    cases = []
    cases.append(("uniform", rng.uniform(0, 1024, (n, 4, 2)).astype(np.float32),
                  rng.uniform(0, 1024, (n, 4, 2)).astype(np.float32),
                  rng.standard_normal((n, 3, 3)).astype(np.float32)))
    torch.manual_seed(0)
    s_int, t_int, *_ = gen["adjust"]("cpu", n)
    g_int = rng.integers(-3, 4, (n, 3, 3)).astype(np.float32)
    g_int[rng.random((n, 3, 3)) < 0.3] = -0.0
    cases.append(("int", s_int.numpy().copy(), t_int.numpy().copy(), g_int))
    ws, wt, _ = wall_problems(n, 31)
    cases.append(("wall", ws.reshape(n, 4, 2), wt.reshape(n, 4, 2),
                  rng.standard_normal((n, 3, 3)).astype(np.float32)))
    es, et = edge_problems()
    ne = es.shape[0]
    cases.append(("edge", es.reshape(ne, 4, 2), et.reshape(ne, 4, 2),
                  rng.standard_normal((ne, 3, 3)).astype(np.float32)))
    pick = lambda *shape: rng.choice(vals, size=shape).astype(np.float32)  # noqa: E731
    cases.append(("special", pick(n, 4, 2), pick(n, 4, 2), pick(n, 3, 3)))
    bits = lambda *shape: rng.integers(0, 2**32 - 1, size=shape, dtype=np.uint32,  # noqa: E731
                                       endpoint=True).view(np.float32)
    cases.append(("bits", bits(n, 4, 2), bits(n, 4, 2), bits(n, 3, 3)))
    f64 = [("f64_uniform", rng.uniform(-512, 512, (n, 4, 2)), rng.uniform(-512, 512, (n, 4, 2)),
            rng.standard_normal((n, 3, 3))),
           ("f64_wall", ws.astype(np.float64).reshape(n, 4, 2), wt.astype(np.float64).reshape(n, 4, 2),
            rng.standard_normal((n, 3, 3))),
           ("f64_edge", es.astype(np.float64).reshape(ne, 4, 2), et.astype(np.float64).reshape(ne, 4, 2),
            rng.standard_normal((ne, 3, 3)))]
    out, names = {}, []
    prev = torch.get_default_dtype()
    try:
        for tag, src, tar, gH in cases + f64:
            torch.set_default_dtype(torch.float64 if src.dtype == np.float64 else torch.float32)
            S = torch.from_numpy(src.copy()).requires_grad_(True)
            T = torch.from_numpy(tar.copy()).requires_grad_(True)
            H = run_ref_statements("ACA_vanilla", bs=src.shape[0], src=S, tar=T)["H"]
            assert H.dtype == S.dtype
            H.backward(torch.from_numpy(gH))
            names.append(tag)
            out.update({f"{tag}_src": src, f"{tag}_tar": tar, f"{tag}_gH": gH,
                        f"{tag}_H": H.detach().numpy().copy(),
                        f"{tag}_gsrc": S.grad.numpy().copy(), f"{tag}_gtar": T.grad.numpy().copy()})
    finally:
        torch.set_default_dtype(prev)
    out["cases"] = np.array(names)
    np.savez_compressed(os.path.join(OUT, "torch_vanilla_grad.npz"), **out)
    return ("torch_vanilla_grad.npz: ATen autograd through the reference's ACA_vanilla statements "
            "on CPU torch %s (ATen CPU capability %s): H, dL/dsrc, dL/dtar for H.backward(gH) on "
            "%s" % (torch.__version__, torch.backends.cpu.get_cpu_capability(), ", ".join(names)))


if __name__ == "__main__":
    if sys.argv[1:] == ["--torch-bcast"]:  # this fixture alone, appended to the manifest
        line = torch_bcast()
        with open(os.path.join(OUT, "MANIFEST.txt"), "a") as f:
            f.write("- " + line + "\n")
        print(line)
    elif sys.argv[1:] == ["--torch-vanilla-grad"]:  # this fixture alone, appended to the manifest
        line = torch_vanilla_grad()
        with open(os.path.join(OUT, "MANIFEST.txt"), "a") as f:
            f.write("- " + line + "\n")
        print(line)
    elif sys.argv[1:] == ["--torch-grad"]:  # this fixture alone, appended to the manifest
        line = torch_rect_grad()
        with open(os.path.join(OUT, "MANIFEST.txt"), "a") as f:
            f.write("- " + line + "\n")
        print(line)
    elif sys.argv[1:] == ["--torch-grad-large"]:  # this fixture alone, appended to the manifest
        line = torch_rect_grad_large()
        with open(os.path.join(OUT, "MANIFEST.txt"), "a") as f:
            f.write("- " + line + "\n")
        print(line)
    elif sys.argv[1:] == ["--torch-f64"]:  # this fixture alone, appended to the manifest
        line = torch_aca_f64()
        with open(os.path.join(OUT, "MANIFEST.txt"), "a") as f:
            f.write("- " + line + "\n")
        print(line)
    elif sys.argv[1:] == ["--torch-special"]:  # this fixture alone, appended to the manifest
        line = torch_special()
        with open(os.path.join(OUT, "MANIFEST.txt"), "a") as f:
            f.write("- " + line + "\n")
        print(line)
    else:
        main()
