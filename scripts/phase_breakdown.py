"""Per-phase kernel time of one bench batch from a rocprofv3 trace (rocpd .db):
encode (pixel prep .. pack_unet_input), 20 steps, decode (after the last DDIM ..
paste_back).  Uses the first batch that has `nsteps` DDIM kernels in a row."""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = sorted(c.execute("select name, start, end from kernels"), key=lambda r: r[1])
    kind = lambda r: "enc0" if "prep_pixels" in r[0] else "pack" if "pack_unet_input" in r[0] else \
        "ddim" if "ddim_cfg_kernel" in r[0] else "paste" if "paste_back" in r[0] else None
    marks = [(i, kind(r)) for i, r in enumerate(rows) if kind(r)]
    for a in range(len(marks)):
        if marks[a][1] != "enc0":
            continue
        seq = [m for m in marks[a:] if m[1] != "enc0"][: nsteps + 2]
        if len(seq) == nsteps + 2 and seq[0][1] == "pack" and all(m[1] == "ddim" for m in seq[1:-1]) \
                and seq[-1][1] == "paste":
            enc = rows[marks[a][0]:seq[0][0] + 1]
            steps = rows[seq[0][0] + 1:seq[-2][0] + 1]
            dec = rows[seq[-2][0] + 1:seq[-1][0] + 1]
            break
    else:
        sys.exit("no complete batch found")
    tot = 0.0
    for name, seg in (("encode", enc), ("steps", steps), ("decode", dec)):
        dur = sum(e - s for _, s, e in seg) / 1e6
        tot += dur
        print(f"== {name}: {len(seg)} kernels, busy {dur:.2f} ms, wall {(seg[-1][2] - seg[0][1]) / 1e6:.2f} ms")
        if name == "steps":
            continue
        agg = collections.defaultdict(lambda: [0, 0])
        for n, s, e in seg:
            k = n.split("(")[0]
            agg[k][0] += e - s
            agg[k][1] += 1
        for k, (t, n) in sorted(agg.items(), key=lambda x: -x[1][0])[:12]:
            print(f"  {t / 1e6:8.3f} ms n={n:4d} {k}")
    print(f"batch busy {tot:.2f} ms")


if __name__ == "__main__":
    main()
