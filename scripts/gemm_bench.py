"""Micro-benchmark of ls_conv2d on the UNet's contraction shapes (HIP events,
median of N launches).  usage: python scripts/gemm_bench.py [regstage] [tile]"""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops, _lib
from latentsync_amd.packing import pack_weight

lib = _lib.load()
SHAPES = [  # (name, n_img, H, Cin, Cout, ksize, act)
    ("conv0 320->320 3x3", 16, 32, 320, 320, 3, 0), ("conv1 640->640 3x3", 16, 16, 640, 640, 3, 0),
    ("conv2 1280 3x3", 16, 8, 1280, 1280, 3, 0), ("conv3 1280 3x3 4x4", 16, 4, 1280, 1280, 3, 0),
    ("conv up0 960->320", 16, 32, 960, 320, 3, 0),
    ("qkv0 320->960", 16, 32, 320, 960, 1, 0), ("geglu0 320->2560", 16, 32, 320, 2560, 1, 1),
    ("ff2_0 1280->320", 16, 32, 1280, 320, 1, 0), ("out0 320->320", 16, 32, 320, 320, 1, 0),
    ("geglu1 640->5120", 16, 16, 640, 5120, 1, 1), ("ff2_1 2560->640", 16, 16, 2560, 640, 1, 0),
    ("geglu2 1280->10240", 16, 8, 1280, 10240, 1, 1), ("ff2_2 5120->1280", 16, 8, 5120, 1280, 1, 0),
    ("qkv2 1280->3840", 16, 8, 1280, 3840, 1, 0), ("plain0 320->2560", 16, 32, 320, 2560, 1, 0), ("vae conv 128 256^2", 16, 256, 128, 128, 3, 0),
    ("vae conv 512 32^2", 16, 32, 512, 512, 3, 0), ("vae conv 512 64^2", 16, 64, 512, 512, 3, 0),
    ("vae conv 256>512 64^2", 16, 64, 256, 512, 3, 0), ("vae conv 256 128^2", 16, 128, 256, 256, 3, 0),
    ("vae conv 128>256 128^2", 16, 128, 128, 256, 3, 0),
    ("out1 640->640", 16, 16, 640, 640, 1, 0), ("out2 1280->1280", 16, 8, 1280, 1280, 1, 0),
    ("sc2a 640->1280", 16, 8, 640, 1280, 1, 0), ("sc2b 1920->1280", 16, 8, 1920, 1280, 1, 0),
    ("sc2c 2560->1280", 16, 8, 2560, 1280, 1, 0), ("out3 1280->1280 4x4", 16, 4, 1280, 1280, 1, 0),
    ("ff2_3 5120->1280 4x4", 16, 4, 5120, 1280, 1, 0), ("sc3 2560->1280 4x4", 16, 4, 2560, 1280, 1, 0),
]


TORCH_REF = False


def run(tag, reps=20, scale=1):
    tot_f, tot_t = 0.0, 0.0
    only = os.environ.get("GEMM_ONLY")  # comma-separated name substrings
    for name, n, H, cin, cout, ks, act in SHAPES:
        if only and not any(o in name for o in only.split(",")):
            continue
        n = n * scale
        x = torch.randn(n, H, H, cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(cout, cin, ks, ks) / (cin * ks * ks) ** 0.5
        pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(cout, device="cuda"), cin, ks, cout,
                        geglu=act == 1)
        kw = {}
        epi = os.environ.get("GEMM_EPI", "")  # side inputs of the UNet's epilogues: res,rowvec,ln
        if "res" in epi and act != 1:
            kw["res"] = torch.randn(n, H, H, cout, device="cuda").to(torch.bfloat16)
        if "rowvec" in epi:
            kw["rowvec"] = (torch.randn(n // 16, pw.N, device="cuda"), 16 * H * H, pw.N)
        if "aff" in epi and ks == 3:  # GroupNorm affine + SiLU on the input (halo conv fuses it)
            kw["aff"] = (torch.rand(n, cin, device="cuda") + 0.5, torch.randn(n, cin, device="cuda") * 0.1, 1, True)
            kw["aff_materialize"] = True
        if "ln" in epi and ks == 1 and cin <= 2048:
            pw.colsum = pw.w.float().sum(1).contiguous()
            kw["ln_stats"] = ops.row_stats(x.view(-1, cin))
        if TORCH_REF:  # vendor library (hipBLASLt via torch.matmul) on the same GEMM: M x K @ K x N
            xa = torch.randn(n * H * H, cin * ks * ks, device="cuda").to(torch.bfloat16)
            wb = torch.randn(cin * ks * ks, cout, device="cuda").to(torch.bfloat16)
            out = torch.empty(n * H * H, cout, device="cuda", dtype=torch.bfloat16)
            launch = lambda: torch.matmul(xa, wb, out=out)
        else:
            out = ops.conv(x, pw, act=act, **kw)
            launch = lambda: ops.conv(x, pw, act=act, out=out, **kw)
        launch()
        torch.cuda.synchronize()
        # graph of 10 launches: GPU time without host submission gaps
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
            e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        t = statistics.median(ts)
        fl = 2.0 * n * H * H * cout * cin * ks * ks
        tot_f += fl; tot_t += t
        print(f"{tag:10s} {name:24s} M={n*H*H:7d} N={cout:6d} K={cin*ks*ks:6d}  {t*1e3:8.1f} us  {fl/t/1e9:7.1f} TF/s")
    print(f"{tag:10s} TOTAL {tot_t:.3f} ms  {tot_f/tot_t/1e9:.1f} TF/s")


if __name__ == "__main__":
    # modes: dma reg nomfma nodma bk32 t1..t6 (forced tile id); suffix @4 = 4x the frames
    for arg in sys.argv[1:] or ["dma"]:
        mode, _, sc = arg.partition("@")
        # mode parts joined by '+': reg, bk32, tN (forced tile id), abN (ablation bits), nomfma, nodma
        parts = mode.split("+")
        ab = {"nomfma": 1, "nodma": 2}.get(mode, 0)
        ab |= sum(int(p[2:]) for p in parts if p.startswith("ab"))
        tile = [int(p[1:]) for p in parts if p.startswith("t") and p[1:].isdigit()]
        lib.ls_set_tuning(1, 1 if "reg" in parts else 0)
        lib.ls_set_tuning(4, ab)
        lib.ls_set_tuning(5, 32 if "bk32" in parts else 64)
        lib.ls_set_tuning(2, tile[0] if tile else 0)
        lib.ls_set_tuning(6, 0 if "norb" in parts else 1)
        lib.ls_set_tuning(8, 0 if "nohalo" in parts else 1)
        lib.ls_set_tuning(10, 1 if "t256" in parts else 0)
        lib.ls_set_tuning(11, 1 if "rs" in parts else 0)
        lib.ls_set_tuning(12, 0 if "nohrp" in parts else 1)
        lib.ls_set_tuning(13, 1 if "bn128" in parts else 0)
        lib.ls_set_tuning(14, 1 if "areg" in parts else 0)
        TORCH_REF = "torch" in parts
        run(arg, scale=int(sc or 1))
