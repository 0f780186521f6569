"""Regenerate the kernel tables of profiles/rNN_profiles.md from the summaries
(prof_summary.py / prof_stream_summary.py outputs).  The header paragraph of
the existing file is kept.
Usage: python3 scripts/dev/profiles_md.py profiles/r05"""
import json
import sys

pre = sys.argv[1]
d = json.load(open(pre + '_stream_pmc_summary.json'))
c2 = json.load(open(pre + '_c2_independent_summary.json'))
old = open(pre + '_profiles.md').read()
out = [old.split('## C2 independent')[0].rstrip() + '\n', '## C2 independent (bench.py headline)\n']
alg = 536857656
out.append(f"encode_independent_kernel, 4096 x 64 KiB per launch: {c2['avg_ns_full_batch'] / 1e3:.1f} us (full-batch "
           f"launches), HBM {c2['hbm_traffic_bytes_per_launch'] / 1e6:.0f} MB per launch (algorithmic: 268 MB read + "
           f"268 MB written = 537 MB, ratio {c2['hbm_traffic_bytes_per_launch'] / alg:.2f}), "
           f"{c2['hbm_GBps_full_batch']:.0f} GB/s.\n")
for c in ['c2s', 'c4', 'c5', 'c5lru', 'c5pair', 'c5dense']:
    if c not in d:
        continue
    v = d[c]
    dev = sum(x['us'] for k, x in v['kernels'].items() if 'rocclr' not in k)
    out += [f'## {c} (device kernels {dev:.0f} us, staging copies excluded)\n',
            '| kernel | launches | us | avg us | HBM MB / launch | GB/s | wait frac |', '|---|---|---|---|---|---|---|']
    rows = [(k, x) for k, x in v['kernels'].items() if 'rocclr' not in k][:6]
    for k, x in rows:
        out.append(f"| {k} | {x['launches']} | {x['us']:.1f} | {x['avg_us']:.1f} | "
                   f"{x['hbm_bytes_per_launch'] / 1e6:.1f} | {x['hbm_GBps']:.1f} | {x.get('wait_any_frac')} |")
    if c == 'c2s' and 'c2s_seeded' in d:
        s = d['c2s_seeded']
        out.append(f"\nc2s_seeded (the seeded stream parse the bench times): {s['us_sum']:.1f} us, HBM "
                   f"{s['hbm_bytes'] / 1e6:.0f} MB (algorithmic 404 MB: ratio {s['hbm_bytes'] / 403621176:.2f}), "
                   f"{s['hbm_GBps']:.0f} GB/s, wait frac {s['wait_any_frac']}.")
    out.append('')
open(pre + '_profiles.md', 'w').write('\n'.join(out) + '\n')
