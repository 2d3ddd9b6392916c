"""The build's spill guard covers every kernel that paces its DMA with a counted
`s_waitcnt vmcnt(N)`, N != 0 (latentsync_amd/build.py COUNTED_VMCNT): a VGPR spill adds
scratch loads/stores to the vmcnt queue and silently breaks such a count, so the build must
refuse a spill in exactly these kernels.  Static check of csrc/ (no compiler, no GPU)."""
import os
import re

from latentsync_amd.build import COUNTED_VMCNT, CSRC

_KERNEL = re.compile(r"__global__\s+void\s+(?:__launch_bounds__\([^\n]*?\)\s+)?(\w+_kernel)\s*\(")
_WAIT = re.compile(r"\b(?:attn_)?wait_vm<([^>]+)>\s*\(\s*\)")


def _counted_waits():
    """{kernel name: [counted wait expressions]} over csrc/*.hip; a wait that precedes every
    kernel of its file (a device helper) is keyed 'helper:<file>'."""
    found = {}
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith(".hip"):
            continue
        src = open(os.path.join(CSRC, f)).read()
        starts = [(m.start(), m.group(1)) for m in _KERNEL.finditer(src)]
        for m in _WAIT.finditer(src):
            n = m.group(1).strip()
            if n == "0":
                continue
            owner = f"helper:{f}"
            for pos, name in starts:
                if pos < m.start():
                    owner = name
            found.setdefault(owner, []).append(n)
    return found


def test_every_counted_wait_kernel_is_spill_guarded():
    found = _counted_waits()
    assert found, "the scan found no counted waits at all (regex out of date?)"
    helpers = [k for k in found if k.startswith("helper:")]
    assert not helpers, f"counted vmcnt waits outside a kernel (attribute them to their callers): {helpers}"
    missing = sorted(k for k in found if not any(g in k for g in COUNTED_VMCNT))
    assert not missing, f"kernels with counted vmcnt waits missing from build.COUNTED_VMCNT: {missing}"


def test_guard_names_exist():
    """No stale names: every COUNTED_VMCNT entry is a kernel defined in csrc/."""
    src = "".join(open(os.path.join(CSRC, f)).read() for f in os.listdir(CSRC) if f.endswith(".hip"))
    names = set(_KERNEL.findall(src))
    assert set(COUNTED_VMCNT) <= names, sorted(set(COUNTED_VMCNT) - names)


def test_known_counted_kernels_detected():
    """The scan itself: the shipped DMA-paced kernels are all found."""
    found = _counted_waits()
    for k in ("conv_gemm_dma_kernel", "gemm_rowblock_kernel", "conv3x3_halo_kernel", "tattn_fused_kernel",
              "attn5_kernel"):
        assert k in found, k
