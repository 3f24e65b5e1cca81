"""Per-op timing of the fused U-Net kernel from MPCD_FUSED_PROF=<file> (wave 0's s_memtime stamps of the first
workgroups of one denoise step): GEMM, statistics, epilogue (+ halo + barrier) per op, averaged over workgroups."""
import sys

import numpy as np

KIND = {0: "same5", 1: "down3", 2: "up4", 3: "pw1", 4: "restore"}
EPI = {0: "bias", 1: "gn", 2: "gn+cond", 3: "gn+res", 4: "eps"}

with open(sys.argv[1], "rb") as f:
    wgs, n_ops = np.frombuffer(f.read(8), dtype=np.int32)
    t = np.frombuffer(f.read(8 * wgs * n_ops * 4), dtype=np.uint64).reshape(wgs, n_ops, 4).astype(np.int64)
    info = np.frombuffer(f.read(4 * 8 * n_ops), dtype=np.int32).reshape(n_ops, 8)
ok = (t[:, :, 0] > 0).all(axis=1) & (t[:, :, 3] > 0).all(axis=1)
t = t[ok]
gemm = np.where(t[:, :, 1] > 0, t[:, :, 1] - t[:, :, 0], 0).mean(axis=0)
stat = np.where(t[:, :, 2] > 0, t[:, :, 2] - t[:, :, 1], 0).mean(axis=0)
epi = np.where(t[:, :, 2] > 0, t[:, :, 3] - t[:, :, 2], t[:, :, 3] - t[:, :, 0]).mean(axis=0)
tot = (t[:, :, 3] - t[:, :, 0]).mean(axis=0)
print(f"{ok.sum()} workgroups; cycles per op (s_memtime ticks)")
print(f"{'op':>3} {'kind':>7} {'epi':>8} {'cinp':>5} {'cout':>5} {'L':>4} {'kc':>3} {'tiles':>5} {'gemm':>8} {'stats':>8} "
      f"{'epi':>8} {'total':>8}")
for i in range(n_ops):
    k, e, ci, co, lo, kc, ntw, ncw = info[i]
    print(f"{i:>3} {KIND[k]:>7} {EPI.get(e, '-'):>8} {ci:>5} {co:>5} {lo:>4} {kc:>3} {f'{ntw}x{ncw}':>5} {gemm[i]:>8.0f} "
          f"{stat[i]:>8.0f} {epi[i]:>8.0f} {tot[i]:>8.0f}")
whole = (t[:, -1, 3] - t[:, 0, 0]).mean()
print(f"sum gemm {gemm.sum():.0f}  stats {stat.sum():.0f}  epi {epi.sum():.0f}  ops {tot.sum():.0f}  first->last {whole:.0f}")
