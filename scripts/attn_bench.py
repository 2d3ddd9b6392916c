"""Attention micro-benchmark on the UNet's shapes (graph-timed, 8 windows):
python scripts/attn_bench.py   (LS_ATTN_V1=1 forces the 16-query kernel)."""
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops

W = int(os.environ.get("WINDOWS", "8"))
CASES = [  # name, batch(frames), tokens, keys, heads, d, kind
    ("spatial L0 d40", 16 * W, 1024, 1024, 8, 40, "self"), ("spatial L1 d80", 16 * W, 256, 256, 8, 80, "self"),
    ("spatial L2 d160", 16 * W, 64, 64, 8, 160, "self"), ("cross L0 d40", 16 * W, 1024, 50, 8, 40, "cross"),
    ("cross L1 d80", 16 * W, 256, 50, 8, 80, "cross"), ("temporal L0 d40", W, 1024, 16, 8, 40, "temporal"),
    ("temporal L1 d80", W, 256, 16, 8, 80, "temporal"),
    ("cross L2 d160", 16 * W, 64, 50, 8, 160, "cross"), ("cross L3 d160", 16 * W, 16, 50, 8, 160, "cross"),
    ("spatial L3 d160", 16 * W, 16, 16, 8, 160, "self"), ("temporal L2 d160", W, 64, 16, 8, 160, "temporal"),
]
if os.environ.get("CFG4"):  # configs[4]: 64^2 latent (WINDOWS windows of 16 frames)
    CASES = [("c4 spatial L0 d40", 16 * W, 4096, 4096, 8, 40, "self"),
             ("c4 spatial L1 d80", 16 * W, 1024, 1024, 8, 80, "self"),
             ("c4 spatial L2 d160", 16 * W, 256, 256, 8, 160, "self")]
if os.environ.get("VAE"):  # SD-VAE mid attention: 1 head, d = 512, 32x32 (256^2) / 64x64 (512^2) latents
    CASES = [("vae mid 32^2 d512", 32 * W, 1024, 1024, 1, 512, "self"),
             ("vae mid 64^2 d512", 4 * W, 4096, 4096, 1, 512, "self")]
FP8 = bool(os.environ.get("ATTN_FP8"))  # self attention through ls_attention_fp8


def run():
    only = os.environ.get("ATTN_ONLY")
    for name, n, N, Nk, heads, d, kind in CASES:
        if only and only not in name:
            continue
        C = heads * d
        if kind == "temporal":
            Fr, S = 16, N
            qkv = torch.randn(n * Fr * S, 3 * C, device="cuda").to(torch.bfloat16)
            o = torch.empty(n * Fr * S, C, device="cuda", dtype=torch.bfloat16)
            st = (Fr * S * 3 * C, 3 * C, S * 3 * C, d)
            f = lambda: ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=n * S, z2=S, heads=heads, nq=Fr,
                                      nk=Fr, head_dim=d, qs=st, ks=st, vs=st, os_=(Fr * S * C, C, S * C, d))
            flops = 4.0 * n * S * heads * Fr * Fr * d
        else:
            q = torch.randn(n * N, C, device="cuda").to(torch.bfloat16)
            kv = torch.randn(n * Nk, 2 * C, device="cuda").to(torch.bfloat16)
            o = torch.empty_like(q)
            f = lambda: ops.attention(q, kv, kv[:, C:], o, batch=n, z2=1, heads=heads, nq=N, nk=Nk, head_dim=d,
                                      qs=(N * C, 0, C, d), ks=(Nk * 2 * C, 0, 2 * C, d),
                                      vs=(Nk * 2 * C, 0, 2 * C, d), os_=(N * C, 0, C, d),
                                      fp8=FP8 and kind == "self" and d in (40, 80))
            flops = 4.0 * n * heads * N * Nk * d
        f()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(5):
                    f()
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 5)
        t = statistics.median(ts)
        print(f"{'fp8' if FP8 and kind == 'self' else os.environ.get('LS_ATTN_V1', 'v2'):3s} {name:18s} {t*1e3:9.1f} us {flops/t/1e9:8.1f} TF/s")
        if kind != "temporal" and not os.environ.get("NO_SDPA"):  # torch SDPA (vendor flash attention) on the same problem, (B, H, N, d)
            qt = torch.randn(n, heads, N, d, device="cuda", dtype=torch.bfloat16)
            kt = torch.randn(n, heads, Nk, d, device="cuda", dtype=torch.bfloat16)
            vt = torch.randn(n, heads, Nk, d, device="cuda", dtype=torch.bfloat16)
            sd = lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt, vt)
            sd()
            torch.cuda.synchronize()
            ts = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); sd(); e1.record(); torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = statistics.median(ts)
            print(f"sdp {name:18s} {t*1e3:9.1f} us {flops/t/1e9:8.1f} TF/s")


run()
