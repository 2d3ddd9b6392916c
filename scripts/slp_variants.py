"""Build the A/B libraries of the gfx950 SLP investigation:

  slp     ls_gemm.hip with SLP vectorisation on (the build that produced wrong
          LayerNorm-folded row-block rows), everything else as shipped;
  slp_bw  slp + every hand-written `s_waitcnt vmcnt(N)` of ls_gemm.hip replaced by
          __builtin_amdgcn_s_waitcnt (an S_WAITCNT the compiler's own waitcnt pass
          sees), i.e. no inline asm the compiler cannot reason about;
  slp_noasm  slp_bw + the row-block kernel's remaining inline asm (lgkmcnt waits and
          compiler memory barriers around s_barrier) replaced by __syncthreads(): the
          kernel then holds no hand-written asm at all;
  slp_nop slp + `-mllvm -amdgpu-snop-padding=4` (s_nop 4 before every instruction);
  slp_wz  slp + `-mllvm -amdgpu-waitcnt-forcezero` (every wait drains all counters);
  slp_sb  slp + a scheduling barrier right after the row-block LayerNorm loop, so
          the packed normalisation stays ahead of the first chunk's LDS reads/MFMAs
          instead of being interleaved with them.

Each goes to latentsync_amd/libls_hip_<name>.so; select with LS_HIP_LIB.  The
disassembly of each row-block LN kernel is written beside it (build/slp/<name>.s).
usage: python scripts/slp_variants.py"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "latentsync_amd", "csrc")
OUT = os.path.join(ROOT, "build", "slp")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result", "-munsafe-fp-atomics"]
HIPCC = "/opt/rocm/bin/hipcc"

WAIT_ASM = 'template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }'
# gfx9 S_WAITCNT simm16: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]; others at max
WAIT_BUILTIN = ("template <int N> __device__ __forceinline__ void wait_vm() "
                "{ __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70); }")
LN_END = "  wait_vm<0>();\n  __builtin_amdgcn_s_barrier();\n  asm volatile(\"\" ::: \"memory\");\n\n  f32x4 acc0[FM][FN]"


def variant(name, src, extra=()):
    top = os.path.join(OUT, name)
    shutil.rmtree(top, ignore_errors=True)
    d = os.path.join(top, "pkg", "csrc")  # csrc/../../include/ls_hip.h resolves as in-tree
    shutil.copytree(CSRC, d)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    with open(os.path.join(d, "ls_gemm.hip"), "w") as f:
        f.write(src)
    objs = []
    procs = []
    for fn in sorted(os.listdir(d)):
        if not fn.endswith(".hip"):
            continue
        flags = FLAGS + (list(extra) if fn == "ls_gemm.hip" else ["-fno-slp-vectorize"])
        o = os.path.join(d, fn[:-4] + ".o")
        procs.append(subprocess.Popen([HIPCC] + flags + ["-c", os.path.join(d, fn), "-o", o]))
        objs.append(o)
    if any(p.wait() for p in procs):
        sys.exit(f"{name}: compile failed")
    lib = os.path.join(ROOT, "latentsync_amd", f"libls_hip_{name}.so")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs)
    # device disassembly of the LN-folded row-block kernel (FLAGS = RB_LN)
    s = subprocess.run([HIPCC] + FLAGS + list(extra) + ["--cuda-device-only", "-S",
                        os.path.join(d, "ls_gemm.hip"), "-o", "-"], capture_output=True, text=True).stdout
    sym = "_ZN2ls20gemm_rowblock_kernelILi10ELi2ELi2ELi1EEEvNS_8ConvArgsE:"
    body = s[s.index(sym):]
    body = body[:body.index(".Lfunc_end", 1)]
    with open(os.path.join(OUT, f"{name}.s"), "w") as f:
        f.write(body)
    print(f"built {lib}: {body.count('v_pk_fma_f32')} v_pk_fma_f32 in the LN row-block kernel", flush=True)


def main():
    only = sys.argv[1:]
    if only:
        global variant
        build = variant
        variant = lambda name, src, extra=(): build(name, src, extra) if name in only else None
    base = open(os.path.join(CSRC, "ls_gemm.hip")).read()
    assert WAIT_ASM in base and base.count(LN_END) == 1
    os.makedirs(OUT, exist_ok=True)
    variant("slp", base)
    variant("slp_bw", base.replace(WAIT_ASM, WAIT_BUILTIN))
    rb_sync = ('    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n    __builtin_amdgcn_s_barrier();\n'
               '    asm volatile("" ::: "memory");\n  };')
    ln_sync = '  __builtin_amdgcn_s_barrier();\n  asm volatile("" ::: "memory");\n\n  f32x4 acc0[FM][FN]'
    assert base.count(rb_sync) == 1 and base.count(ln_sync) == 1
    noasm = base.replace(WAIT_ASM, WAIT_BUILTIN).replace(rb_sync, "    __syncthreads();\n  };")
    variant("slp_noasm", noasm.replace(ln_sync, "  __syncthreads();\n\n  f32x4 acc0[FM][FN]"))
    # compiler-side knobs on the unchanged source: 4 wait states before every
    # instruction (a VALU / MFMA hazard that needs more nops than the compiler
    # inserts disappears), and every s_waitcnt forced to zero (a memory-counter race
    # disappears)
    variant("slp_nop", base, ["-mllvm", "-amdgpu-snop-padding=4"])
    variant("slp_wz", base, ["-mllvm", "-amdgpu-waitcnt-forcezero"])
    variant("slp_sb", base.replace(LN_END, LN_END.replace("  wait_vm<0>();\n", "  __builtin_amdgcn_sched_barrier(0);\n  wait_vm<0>();\n", 1)))


if __name__ == "__main__":
    main()
