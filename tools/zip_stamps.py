"""Per-workgroup phase timing of the fused fp32 zipper's step kernel (k_zstep, zip32.hip) from XRS_ZIP_STAMPS=1
stderr lines: duration per phase, per XCD, and by how many workgroups shared the CU.
    XRS_ZIP_STAMPS=1 python tools/dot32_one.py 3 2> stamps.txt; python tools/zip_stamps.py stamps.txt"""
import collections
import sys

rows = []
for line in open(sys.argv[1]):
    if line.startswith("[zip stamps]"):
        f = line.split()[2:]
        rows.append([int(x) for x in f])
# keep the last call's steps (the file holds every call): group by step, take the last occurrence of each wg
last = {}
for r in rows:
    last[(r[0], r[1])] = r
steps = sorted({k[0] for k in last})
for s in steps:
    wgs = [v for k, v in last.items() if k[0] == s]
    t0 = min(v[3] for v in wgs)
    cu = collections.Counter()
    for v in wgs:
        hw = v[2] & 0xFFFFFFFF
        cu[(v[2] >> 32, (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 0x7)] += 1   # xcc, cu, sh, se (gfx9 HW_ID)
    by = collections.defaultdict(list)
    for v in wgs:
        hw = v[2] & 0xFFFFFFFF
        key = (v[2] >> 32, (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 0x7)
        by[cu[key]].append(v)
    print(f"step {s}: {len(wgs)} workgroups, span {(max(v[7] for v in wgs) - t0) / 1e3:.1f} kcycles (s_memtime: shader clock)")
    for share, vs in sorted(by.items()):
        n = len(vs)
        ph = [sum(v[3 + i + 1] - v[3 + i] for v in vs) / n / 1e3 for i in range(4)]
        st = sum(v[3] - t0 for v in vs) / n / 1e3
        tot = sum(v[7] - v[3] for v in vs) / n / 1e3
        print(f"  {n:4d} wgs sharing a CU {share}x: start +{st:6.2f}, phase1 {ph[0]:6.2f}, T {ph[1]:5.2f}, phase2 {ph[2]:6.2f}, store {ph[3]:5.2f}, total {tot:6.2f} kcycles")
