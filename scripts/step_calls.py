"""Per-call HIP-event table of one UNet denoising step (eager launches, same
kernels as the captured graph): every ls_conv2d / ls_attention / GroupNorm /
LayerNorm call with its shape, time and TF/s, aggregated by shape.

    python scripts/step_calls.py [windows] [resolution]
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from latentsync_amd import ops  # noqa: E402
from latentsync_amd.config import STAGE2_MODEL  # noqa: E402
from latentsync_amd.pipeline import WindowEngine, load_fixed_mask  # noqa: E402
from latentsync_amd.scheduler import DDIMScheduler  # noqa: E402
from latentsync_amd.unet import UNet3DConditionModel  # noqa: E402
from latentsync_amd.vae import AutoencoderKL  # noqa: E402


def main():
    nw = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    phase = sys.argv[3] if len(sys.argv) > 3 else "step"  # step | encode | decode
    dev = torch.device("cuda", 0)
    unet = UNet3DConditionModel(**STAGE2_MODEL).init_weights(41).to(dev).eval()
    vae = AutoencoderKL().init_weights(51).to(dev)
    eng = WindowEngine(unet, vae, DDIMScheduler(**bench.SCHED_CFG), 16, R, 20, 1.0, use_graphs=False, windows=nw)
    faces, audio, init, em, er = bench.synthetic_window(16 * nw, R, R // 8, 384, 1000, dev)
    eng.load(faces, load_fixed_mask(R).to(dev), audio, init, em, er)
    eng._encode()
    eng._step()
    torch.cuda.synchronize()
    recs = []

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        return e

    names = ["conv", "attention", "group_norm", "group_norm_apply", "row_stats", "layer_norm", "feedforward",
             "temporal_attention", "cross_attention_block", "ff_chain", "small_linear", "ddim_cfg_step", "add_rows"]
    names = [n for n in names if hasattr(ops, n)]
    orig = {n: getattr(ops, n) for n in names}

    def wrap(n):
        def f(*a, **kw):
            e0 = ev()
            r = orig[n](*a, **kw)
            e1 = ev()
            nb = 0.0  # algorithmic HBM bytes (operands once, output once)
            if n == "conv":
                x, pw = a[0], a[1]
                x2 = kw.get("x2")
                cin = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
                y = r
                M = y.shape[0] * y.shape[1] * y.shape[2]
                fl = 2.0 * M * pw.N * cin * pw.ksize ** 2
                nb = (x.numel() + (x2.numel() if x2 is not None else 0) + pw.w.numel()) * 2 + y.numel() * y.element_size()
                if kw.get("res") is not None:
                    nb += y.numel() * 2
                key = (n, f"M={M} N={pw.N} K={cin * pw.ksize ** 2} ks={pw.ksize} act={kw.get('act', 0)} "
                          f"res={int(kw.get('res') is not None)} ln={int(kw.get('ln_stats') is not None)} "
                          f"aff={int(kw.get('aff') is not None)} up={int(kw.get('upsample', False))} s={kw.get('stride', 1)}")
            elif n == "attention":
                fl = 4.0 * kw["batch"] * kw["heads"] * kw["nq"] * kw["nk"] * kw["head_dim"]
                hd = kw["heads"] * kw["head_dim"] * kw["batch"] * 2
                nb = hd * (2 * kw["nq"] + 2 * kw["nk"])
                key = (n, f"b={kw['batch']} h={kw['heads']} nq={kw['nq']} nk={kw['nk']} d={kw['head_dim']}")
            elif n == "feedforward":
                x2d, w1, w2 = a[0], a[2], a[3]
                rows, C = x2d.shape
                fl = 2.0 * rows * w1.N * C + 2.0 * rows * w2.N * (w1.N // 2)
                nb = rows * C * 2 * 2 + (w1.w.numel() + w2.w.numel()) * 2
                key = (n, f"rows={rows} C={C} inner={w1.N // 2}")
            elif n == "temporal_attention":
                x2d, pk, ns, F, S = a[0], a[1], a[2], a[3], a[4]
                rows, C = x2d.shape
                fl = 2.0 * rows * 3 * C * C + 4.0 * ns * S * pk.heads * F * F * (C // pk.heads)
                nb = rows * C * 2 * 2
                key = (n, f"rows={rows} C={C} F={F}")
            elif n == "ff_chain":
                o2d, pk = a[0], a[3]
                rows, C = o2d.shape
                fl = 4.0 * rows * C * C + 6.0 * rows * C * pk.inner
                nb = rows * C * 2 * 4 + (pk.w1.numel() + pk.w2.numel() + pk.wo.numel() + pk.wp.numel()) * 2
                key = (n, f"rows={rows} C={C} inner={pk.inner}")
            elif n == "cross_attention_block":
                x2d = a[0]
                rows, C = x2d.shape
                fl = 4.0 * rows * C * C
                nb = rows * C * 2 * 2
                key = (n, f"rows={rows} C={C}")
            elif n == "group_norm":
                # the finalize reads the producer's per-128-row slot sums (2 x C fp32 per slot),
                # not the tensor; only without them is there a read pass over x (| x2)
                fl = 0.0
                x, x2 = a[0], kw.get("x2")
                pps = x.numel() // x.shape[-1] // a[5]
                have = ops._colsums(x, pps) is not None and (x2 is None or ops._colsums(x2, pps) is not None)
                nb = 0.0
                for t in (x, x2):
                    if t is not None:
                        rows = t.numel() // t.shape[-1]
                        nb += (rows // ops.GN_SLOT_ROWS) * 2 * t.shape[-1] * 4 if have else t.numel() * t.element_size()
                key = (n, f"shape={tuple(x.shape)} {'slot sums' if have else 'read pass'}")
            else:
                fl = 0.0
                t0 = a[0] if hasattr(a[0], "numel") else None
                nb = 2.0 * t0.numel() * t0.element_size() if t0 is not None else 0.0
                key = (n, f"shape={tuple(t0.shape) if t0 is not None else ''}")
            recs.append((key, e0, e1, fl, nb))
            return r
        return f

    for n in names:
        setattr(ops, n, wrap(n))
    {"step": eng._step, "encode": eng._encode, "decode": eng._decode}[phase]()
    torch.cuda.synchronize()
    for n in names:
        setattr(ops, n, orig[n])
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    tot = 0.0
    for key, e0, e1, fl, nb in recs:
        t = e0.elapsed_time(e1)
        agg[key][0] += 1
        agg[key][1] += t
        agg[key][2] += fl
        agg[key][3] += nb
        tot += t
    print(f"{phase}: {len(recs)} calls, {tot:.3f} ms summed (windows={nw}, R={R})")
    fam = collections.defaultdict(float)
    for (n, _), (c, t, fl, nb) in agg.items():
        fam[n] += t
    for n, t in sorted(fam.items(), key=lambda x: -x[1]):
        print(f"  {n:22s} {t:8.3f} ms")
    # excess over a practical roofline: max(flops / 1.6 PF/s, bytes / 6 TB/s)
    ideal = lambda fl, nb: max(fl / 1.6e15, nb / 6e12) * 1e3
    print(f"practical roofline (1.6 PF/s MFMA, 6 TB/s HBM): {sum(ideal(v[2], v[3]) for v in agg.values()):.3f} ms "
          f"of {tot:.3f} ms")
    for (n, k), (c, t, fl, nb) in sorted(agg.items(), key=lambda x: -(x[1][1] - ideal(x[1][2], x[1][3]))):
        tf = fl / (t * 1e-3) / 1e12 if fl else 0.0
        gbs = nb / (t * 1e-3) / 1e9
        print(f"{t:8.3f} ms excess {t - ideal(fl, nb):7.3f} n={c:3d} avg {t / c * 1e3:8.1f} us {tf:7.1f} TF/s "
              f"{gbs:6.0f} GB/s  {n:16s} {k}")


if __name__ == "__main__":
    main()
