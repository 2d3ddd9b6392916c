"""Measured dense bf16 GEMM ceiling on the box, and the vendor library beside this
repo's kernels on the UNet's contraction shapes (VERDICT r1 'What's weak' 3).

  * plain square GEMMs (4096^3, 8192^3) through torch.matmul (hipBLASLt) and through
    ls_conv2d (ksize 1: the repo's DMA GEMM) -- the best of them is the ceiling
    bench.py reports as roofline.peak_measured;
  * every distinct UNet conv / linear shape of one step at 16 windows per call:
    ls_conv2d (with its real epilogue) vs torch.matmul on the same M x K x N.

Timing: 10 launches captured in a hipGraph, median of 20 replays, HIP events; random
operands (the clock depends on the data -- MI355X_MICROARCH.md, DVFS give-back).
usage: python scripts/gemm_ceiling.py OUT.json"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import ops  # noqa: E402
from latentsync_amd.packing import pack_weight  # noqa: E402

W16 = 16 * 16  # frames in flight at 16 windows per UNet call
UNET = [  # (name, n_img, H, Cin, Cout, ksize, act)
    ("conv3x3 320 @32^2", W16, 32, 320, 320, 3, 0), ("conv3x3 640 @16^2", W16, 16, 640, 640, 3, 0),
    ("conv3x3 1280 @8^2", W16, 8, 1280, 1280, 3, 0), ("conv3x3 1280 @4^2", W16, 4, 1280, 1280, 3, 0),
    ("conv3x3 2560->1280 @4^2", W16, 4, 2560, 1280, 3, 0), ("conv3x3 960->320 @32^2", W16, 32, 960, 320, 3, 0),
    ("qkv 320->960 @32^2", W16, 32, 320, 960, 1, 0), ("geglu 320->2560 @32^2", W16, 32, 320, 2560, 1, 1),
    ("ff2 1280->320 @32^2", W16, 32, 1280, 320, 1, 0), ("geglu 640->5120 @16^2", W16, 16, 640, 5120, 1, 1),
    ("ff2 2560->640 @16^2", W16, 16, 2560, 640, 1, 0), ("geglu 1280->10240 @8^2", W16, 8, 1280, 10240, 1, 1),
    ("ff2 5120->1280 @8^2", W16, 8, 5120, 1280, 1, 0), ("qkv 1280->3840 @8^2", W16, 8, 1280, 3840, 1, 0),
    ("geglu 1280->10240 @4^2", W16, 4, 1280, 10240, 1, 1),
    ("vae conv3x3 128 @256^2", 32, 256, 128, 128, 3, 0), ("vae conv3x3 256 @128^2", 32, 128, 256, 256, 3, 0),
    ("vae conv3x3 512 @64^2", 32, 64, 512, 512, 3, 0), ("vae conv3x3 512 @32^2", 32, 32, 512, 512, 3, 0),
]


def timed(launch, reps=20):
    launch()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(10):
                launch()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    return statistics.median(ts)  # ms


def torch_gemm(M, K, N):
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    return timed(lambda: torch.matmul(a, b, out=o))


def ours(n, H, cin, cout, ks, act):
    x = torch.randn(n, H, H, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(cout, cin, ks, ks) / (cin * ks * ks) ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(cout, device="cuda"), cin, ks, cout,
                    geglu=act == 1)
    out = ops.conv(x, pw, act=act)
    return timed(lambda: ops.conv(x, pw, act=act, out=out))


def main():
    res = {"square": [], "unet": []}
    best = 0.0
    for S in (4096, 8192):
        fl = 2.0 * S ** 3
        t_t = torch_gemm(S, S, S)
        # ls_conv2d as a linear: S rows = (S images of 1x1), K = S, N = S
        x = torch.randn(S, 1, 1, S, device="cuda").to(torch.bfloat16)
        pw = ops.Packed((torch.randn(S, S, device="cuda") / S ** 0.5).to(torch.bfloat16), None, S, 1, S)
        out = ops.conv(x, pw)
        t_o = timed(lambda: ops.conv(x, pw, out=out))
        r = {"M=N=K": S, "hipblaslt_ms": round(t_t, 4), "hipblaslt_tflops": round(fl / t_t / 1e9, 1),
             "ls_conv2d_ms": round(t_o, 4), "ls_conv2d_tflops": round(fl / t_o / 1e9, 1)}
        best = max(best, r["hipblaslt_tflops"], r["ls_conv2d_tflops"])
        res["square"].append(r)
        print(json.dumps(r), flush=True)
    for name, n, H, cin, cout, ks, act in UNET:
        M, K = n * H * H, cin * ks * ks
        fl = 2.0 * M * cout * K
        t_o = ours(n, H, cin, cout, ks, act)
        t_t = torch_gemm(M, K, cout)
        r = {"shape": name, "M": M, "N": cout, "K": K, "ls_conv2d_us": round(t_o * 1e3, 1),
             "ls_conv2d_tflops": round(fl / t_o / 1e9, 1), "hipblaslt_us": round(t_t * 1e3, 1),
             "hipblaslt_tflops": round(fl / t_t / 1e9, 1)}
        res["unet"].append(r)
        print(json.dumps(r), flush=True)
    res["best_tflops"] = best
    res["note"] = ("dense bf16 GEMM ceiling measured on this MI355X: best of hipBLASLt (torch.matmul) and "
                   "ls_conv2d on square 4096^3 / 8192^3, random operands; spec dense peak 2500 TF/s")
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
