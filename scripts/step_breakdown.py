"""Break a rocprofv3 kernel trace down per UNet step (between DDIM kernels)."""
import collections, csv, sqlite3, sys


def load(path):
    if path.endswith(".db"):  # rocprofv3 default (rocpd sqlite) output
        c = sqlite3.connect(path)
        return [dict(Kernel_Name=n, Start_Timestamp=s, End_Timestamp=e, Grid_Size_X=g)
                for n, s, e, g in c.execute("select name, start, end, grid_x from kernels")]
    return list(csv.DictReader(open(path)))


def main():
    rows = load(sys.argv[1])
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if 'ddim_cfg_kernel' in r['Kernel_Name']]
    k = len(idx) // 2
    seg = rows[idx[k] + 1:idx[k + 1] + 1]
    dur = lambda r: int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    t0, t1 = int(seg[0]['Start_Timestamp']), int(seg[-1]['End_Timestamp'])
    print('step wall ms', (t1 - t0) / 1e6, 'busy ms', sum(map(dur, seg)) / 1e6, 'kernels', len(seg))
    agg = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        n = r['Kernel_Name'].split('(')[0]
        agg[n][0] += dur(r); agg[n][1] += 1
    for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:16]:
        print(f"{t/1e6:8.3f} ms  n={c:4d} avg {t/c/1e3:7.1f}us {n}")
    agg2 = collections.defaultdict(list)
    gemm = lambda n: 'conv_gemm' in n or 'gemm_rowblock' in n or 'conv3x3_halo' in n  # the ls_conv2d kernels
    for r in seg:
        if gemm(r['Kernel_Name']):
            agg2[(r['Kernel_Name'].split('(')[0].replace('void ls::conv_gemm_kernel', ''), r['Grid_Size_X'])].append(dur(r))
    fam = [dur(r) for r in seg if gemm(r['Kernel_Name']) or 'splitk_reduce' in r['Kernel_Name']]
    ncall = sum(gemm(r['Kernel_Name']) for r in seg)
    print(f"conv_gemm family: {ncall} ls_conv2d calls (+{len(fam) - ncall} split-K reduces), total {sum(fam)/1e6:.3f} ms, "
          f"avg per ls_conv2d call {sum(fam)/max(1, ncall)/1e3:.1f} us  (bench.py roofline.avg_launch_ms)")
    att = [dur(r) for r in seg if 'attn' in r['Kernel_Name']]
    print(f"attention kernels: {len(att)} launches, total {sum(att)/1e6:.3f} ms, avg {sum(att)/max(1,len(att))/1e3:.1f} us")
    print('--- gemm shapes')
    for k2, v in sorted(agg2.items(), key=lambda x: -sum(x[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
        print(f"{sum(v)/1e6:7.3f} ms n={len(v):3d} avg {sum(v)/len(v)/1e3:7.1f}us {k2}")


if __name__ == '__main__':
    main()
