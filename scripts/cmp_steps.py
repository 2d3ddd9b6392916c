"""Compare rocprofv3 kernel traces of bench.py: per-kernel time of one mid-run UNet
step (between DDIM kernels).  Each side may be several traces (comma-separated
globs): per kernel the minimum over them is used (drift between runs of a box).
usage: python scripts/cmp_steps.py 'A*' 'B*' [top]"""
import collections
import glob
import os
import sqlite3
import sys


def rows(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(path)
    return sorted(c.execute("select name, start, end from kernels"), key=lambda r: r[1])


def step(rs):
    idx = [i for i, r in enumerate(rs) if "ddim_cfg_kernel" in r[0]]
    k = len(idx) // 2
    seg = rs[idx[k] + 1:idx[k + 1] + 1]
    agg = collections.defaultdict(lambda: [0, 0])
    for n, s, e in seg:
        n = n.split("(")[0]
        agg[n][0] += e - s
        agg[n][1] += 1
    return agg, (seg[-1][2] - seg[0][1]) / 1e6, sum(e - s for _, s, e in rs) / 1e6


def side(spec):
    paths = [p for g in spec.split(",") for p in sorted(glob.glob(g)) if os.path.isdir(p) or p.endswith(".db")]
    steps = [step(rows(p)) for p in paths]
    agg = collections.defaultdict(lambda: [0, 0])
    for n in set().union(*[s[0] for s in steps]):
        agg[n] = min((s[0][n] for s in steps if n in s[0]), key=lambda v: v[0])
    print(f"{spec}: {len(paths)} trace(s), step wall ms " + " ".join(f"{s[1]:.3f}" for s in steps))
    return agg, min(s[1] for s in steps), min(s[2] for s in steps)


def main():
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    (sa, ta, ba), (sb, tb, bb) = side(sys.argv[1]), side(sys.argv[2])
    print(f"step wall ms {ta:.3f} -> {tb:.3f}   all kernels busy ms {ba:.2f} -> {bb:.2f}")
    for n in sorted(set(sa) | set(sb), key=lambda n: -abs(sb[n][0] - sa[n][0]))[:top]:
        print(f"{(sb[n][0] - sa[n][0]) / 1e6:+8.3f} ms  {sa[n][0] / 1e6:8.3f} -> {sb[n][0] / 1e6:8.3f}  n={sb[n][1]:4d} {n}")


if __name__ == "__main__":
    main()
