"""Workgroup residency from gpurun_out/wgtrace_L<layer>.bin (MPCD_UNET_WGTRACE): per CU, how many workgroups
ran at once and how far apart co-resident workgroups started (phase desynchronisation)."""
import sys
from collections import defaultdict

import numpy as np

for path in sys.argv[1:]:
    raw = np.fromfile(path, dtype=np.uint32)
    nb, rb, tile, lds = raw[:4].astype(np.int64)
    t = raw[4:].reshape(-1, 4).astype(np.int64)
    st, en, hw, xcc = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    ok = en != 0
    st, en, hw, xcc = st[ok], en[ok], hw[ok], xcc[ok]
    base = st.min()
    st, en = (st - base) * 0.01, (en - base) * 0.01  # microseconds
    cu = (xcc & 0xF) * 64 + ((hw >> 13) & 0x3) * 16 + ((hw >> 12) & 1) * 8 + ((hw >> 8) & 0xF)
    dur = en - st
    print(f"{path}: {nb} workgroups (rb {rb}, tile {tile // 16}x{tile % 16}, lds {lds}); launch {en.max():.1f} us; "
          f"wg duration mean {dur.mean():.2f} us (p10 {np.percentile(dur, 10):.2f}, p90 {np.percentile(dur, 90):.2f}); "
          f"distinct CUs {len(set(cu.tolist()))}")
    conc, lag = [], []
    for c in sorted(set(cu.tolist()))[:256]:
        m = cu == c
        s, e = st[m], en[m]
        ev = sorted([(x, 1) for x in s] + [(x, -1) for x in e])
        cur = mx = 0
        acc = 0.0
        last = ev[0][0]
        for x, d in ev:
            acc += cur * (x - last)
            last = x
            cur += d
            mx = max(mx, cur)
        conc.append((mx, acc / (e.max() - s.min())))
        ss = np.sort(s)
        lag.append(np.median(np.diff(ss)))
    conc = np.array(conc)
    print(f"  per CU: max co-resident {np.bincount(conc[:, 0].astype(int)).tolist()} (histogram), mean resident "
          f"{conc[:, 1].mean():.2f}; median start spacing {np.median(lag):.2f} us vs wg duration {dur.mean():.2f} us")
