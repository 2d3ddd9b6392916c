"""HBM traffic per ls_conv2d call from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE) of `bench.py --steps 1 --warmup 0 --no-graphs ...`.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md § HBM: FETCH_SIZE /
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced streaming read -- every operand read of the conv_gemm
kernels is a 16-B-per-lane global_load_lds / global_load, so it is doubled;
WRITE_SIZE is exact for 16-B stores (the epilogue's).  One denoising step is
the span between two consecutive ddim_cfg_kernel dispatches (the middle one).

usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    rows = list(csv.DictReader(open(files[0])))
    per = collections.OrderedDict()
    for r in rows:
        did = int(r.get("Dispatch_Id") or r.get("Dispatch_ID") or r["Correlation_Id"])
        name = r["Kernel_Name"]
        val = float(r["Counter_Value"])
        if did not in per:
            per[did] = [name, 0.0]
        per[did][1] += val
    return [(k, v[0], v[1]) for k, v in sorted(per.items())]


def one_step(disp):
    idx = [i for i, (_, n, _) in enumerate(disp) if "ddim_cfg_kernel" in n]
    k = len(idx) // 2
    return disp[idx[k] + 1: idx[k + 1] + 1]


def family(seg):
    fam = lambda n: "conv_gemm" in n or "gemm_rowblock" in n or "conv3x3_halo" in n  # the ls_conv2d kernels
    calls = sum(fam(n) for _, n, _ in seg)
    kib = sum(v for _, n, v in seg if fam(n) or "splitk_reduce" in n)
    return calls, kib


def main():
    fetch, write = one_step(load(sys.argv[1])), one_step(load(sys.argv[2]))
    cf, fk = family(fetch)
    cw, wk = family(write)
    assert cf == cw, (cf, cw)
    fb = 2.0 * fk * 1024 / cf
    wb = wk * 1024 / cw
    attn_f = [v for _, n, v in fetch if "attn" in n]
    attn_w = [v for _, n, v in write if "attn" in n]
    res = {
        "kernel": "conv_gemm family (every ls_conv2d call: tiled / row-block / halo-tile GEMM + split-K reduce), one UNet step",
        "calls": cf,
        "fetch_bytes_per_call": fb, "write_bytes_per_call": wb, "hbm_bytes_per_call": fb + wb,
        "fetch_raw_kib_step": fk, "write_kib_step": wk,
        "attention_hbm_bytes_per_call": (2.0 * sum(attn_f) + sum(attn_w)) * 1024 / max(1, len(attn_f)),
        "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE as is; KiB -> bytes",
        "source": [sys.argv[1], sys.argv[2]],
    }
    out = json.dumps(res, indent=1)
    print(out)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(out + "\n")


if __name__ == "__main__":
    main()
