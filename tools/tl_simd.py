"""Per-SIMD occupancy of a seg-pass timeline (tools/timeline.py .npy with the
XCC id in the high word of the HW_ID record): the time each SIMD spends with
0, 1, 2, 3 resident waves, and the issue capacity lost to SIMDs holding fewer
than two waves (a lone wave issues at about half rate)."""
import sys
import numpy as np


def analyse(path):
    rec = np.load(path)
    t0 = rec[:, 0].min()
    st = (rec[:, 0] - t0) / 100.0
    en = (rec[:, 1] - t0) / 100.0
    hw = rec[:, 2] & 0xffffffff
    xcc = (rec[:, 2] >> 32) & 0xf
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    span = en.max()
    simds = np.unique(key)
    tot = np.zeros(5)
    for k in simds:
        m = key == k
        ev = np.concatenate([np.stack([st[m], np.ones(m.sum())], 1), np.stack([en[m], -np.ones(m.sum())], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        t_prev, c = 0.0, 0
        for t, d in ev:
            tot[min(c, 4)] += t - t_prev
            t_prev, c = t, c + int(d)
        tot[0] += span - t_prev
    frac = tot / (len(simds) * span)
    lost = frac[0] + 0.5 * frac[1]
    return dict(simds=len(simds), span_us=round(span, 1), time_frac_by_resident=[round(x, 4) for x in frac],
                issue_capacity_lost=round(lost, 4))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p, analyse(p))
