"""Builds libls_hip.so (all HIP kernels + the C-ABI) in-tree for gfx950.

    python -m latentsync_amd.build        # incremental
    LS_DIAG_BUILD=1 python -m latentsync_amd.build   # + the measured-and-rejected kernels
Compiles each csrc/*.hip with hipcc --offload-arch=gfx950 -O3 -fPIC into
build/ objects and links latentsync_amd/libls_hip.so.  No CUDA, no dual path.
The default build compiles only the kernels the dispatch uses; the diagnostics build
(-DLS_DIAG_KERNELS, objects in build/obj_diag) adds the A/B variants DESIGN.md section 3
records as measured and rejected (register-staged / A-in-register / phased / 4-stage GEMMs,
the 256x128 3-stage tile, BK 32, attn6) for re-measurement.
"""
import concurrent.futures as cf
import os
import re
import shutil
import subprocess
import sys
import tempfile
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
DIAG = os.environ.get("LS_DIAG_BUILD", "") not in ("", "0")
OBJ = os.path.join(REPO, "build", "obj_diag" if DIAG else "obj")
MODE_STAMP = os.path.join(REPO, "build", "lib_mode")
LIB = os.path.join(HERE, "libls_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -fno-slp-vectorize: no v_pk_*_f32 packed fp32 math.  (1) Beside MFMAs it costs
# issue cycles (MI355X_MICROARCH.md, 'price of one filler').  (2) Correctness: the
# SLP-packed LayerNorm normalisation of the row-block GEMM (v_pk_fma_f32 with
# op_sel picking one half of a VGPR pair whose other half was being recycled)
# produced intermittently wrong values on gfx950 -- second wave of a SIMD, run to
# run different -- and bit-exact results without packing (scripts/debug_rb3.py).
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result", "-munsafe-fp-atomics",
         "-fno-slp-vectorize"] + (["-DLS_DIAG_KERNELS"] if DIAG else [])


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs.append(os.path.join(REPO, "include", "ls_hip.h"))
    return max(os.path.getmtime(h) for h in hdrs)


# Kernels that pace their operand DMA with counted `s_waitcnt vmcnt(N)`: a register
# (VGPR) spill adds scratch loads/stores to the vmcnt queue and silently breaks the count,
# so the build refuses any spill in them (hipcc resource-usage remarks).
# tests/test_build_guards.py checks that every kernel with a non-zero counted wait in csrc/ is listed.
COUNTED_VMCNT = ("gemm_rowblock_kernel", "conv_gemm_dma_kernel", "attn5_kernel", "attn8_kernel", "tattn_fused_kernel",
                 "attnw_kernel", "conv3x3_halo_kernel", "attn6_kernel", "conv_gemm_p8_kernel", "conv_gemm_big4_kernel",
                 "conv_gemm_areg_kernel", "ff_pair_kernel", "ff_chain_kernel")


def _spills(stderr):
    bad, cur = [], None
    for line in stderr.splitlines():
        m = re.search(r"remark: +Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            continue
        m = re.search(r"remark: +VGPRs Spill: (\d+)", line)
        if m and cur and int(m.group(1)) > 0 and any(k in cur for k in COUNTED_VMCNT):
            bad.append(f"{cur}: {line.split('remark:')[1].strip()}")
    return bad


OBJDUMP = os.environ.get("LLVM_OBJDUMP", "/opt/rocm/lib/llvm/bin/llvm-objdump")
# every packed-fp32 VALU opcode (v_pk_fma/mul/add/mov_f32 ...), any op_sel bit set
_PK_OPSEL = re.compile(r"v_pk_\w+_f32\b[^\n]*\bop_sel:\[([01,]+)\]")


def _packed_opsel(obj):
    """Disassembled gfx950 instructions of `obj` of the packed-fp32 op_sel form that
    miscomputes beside MFMAs (see FLAGS); [] when clean.  A missing llvm-objdump, or one that
    cannot extract the gfx950 code object, fails the build unless LS_SKIP_OPSEL_GUARD=1."""
    skip = os.environ.get("LS_SKIP_OPSEL_GUARD", "") not in ("", "0")
    if not os.path.exists(OBJDUMP):
        if skip:
            warnings.warn(f"packed-fp32 op_sel guard skipped (LS_SKIP_OPSEL_GUARD): {OBJDUMP} not found")
            return []
        raise RuntimeError(f"packed-fp32 op_sel guard: {OBJDUMP} not found (LS_SKIP_OPSEL_GUARD=1 to build without it)")
    with tempfile.TemporaryDirectory() as td:
        cp = os.path.join(td, "k.o")
        shutil.copy(obj, cp)
        r = subprocess.run([OBJDUMP, "--offloading", cp], capture_output=True, text=True, cwd=td)
        dev = [f for f in os.listdir(td) if "gfx950" in f]
        if r.returncode != 0 or not dev:
            msg = f"could not extract the gfx950 code object of {obj} ({r.stderr.strip()[:200]})"
            if skip:
                warnings.warn("packed-fp32 op_sel guard skipped (LS_SKIP_OPSEL_GUARD): " + msg)
                return []
            raise RuntimeError("packed-fp32 op_sel guard: " + msg + " (LS_SKIP_OPSEL_GUARD=1 to build without it)")
        r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", os.path.join(td, dev[0])], capture_output=True, text=True)
    return [m.group(0).split("//")[0].strip() for m in _PK_OPSEL.finditer(r.stdout) if "1" in m.group(1)]


def _compile(src, obj, dep_time):
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), dep_time):
        return obj, None
    cmd = [HIPCC] + FLAGS + ["-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, r.stderr
    with open(obj[:-2] + ".remarks", "w") as f:  # per-kernel VGPR / AGPR / occupancy (scripts/kernel_regs.py)
        f.write(r.stderr)
    bad = _spills(r.stderr)
    if bad:
        os.remove(obj)
        return obj, "register spills in counted-vmcnt kernels:\n" + "\n".join(bad)
    try:
        bad = _packed_opsel(obj)
    except RuntimeError as e:
        os.remove(obj)
        return obj, str(e)
    if bad:
        os.remove(obj)
        return obj, f"{len(bad)} packed-fp32 op_sel instructions (wrong beside MFMAs on gfx950), e.g.:\n" + "\n".join(bad[:4])
    return obj, None


def build(verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    dep_time = _deps()
    objs = []
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        futs = [ex.submit(_compile, s, os.path.join(OBJ, os.path.basename(s)[:-4] + ".o"), dep_time) for s in srcs]
        for f in futs:
            obj, err = f.result()
            if err:
                raise RuntimeError(f"hipcc failed for {obj}:\n{err}")
            objs.append(obj)
    mode = "diag" if DIAG else "default"
    old_mode = open(MODE_STAMP).read().strip() if os.path.exists(MODE_STAMP) else "default"
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs) or old_mode != mode:
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr)
        with open(MODE_STAMP, "w") as f:
            f.write(mode + "\n")
        if verbose:
            print("built", LIB, f"({mode})")
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
