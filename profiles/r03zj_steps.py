"""Per chunk step of the LAST traced K-Modes call: durations of assign / decide / apply and the gaps between them."""
import csv
import glob
import sys

import numpy as np

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
# the last call: from the last kmb_ff_persist (or kmb_ff_start) on
last = max(i for i, k in enumerate(ks) if "kmb_ff_start" in k[0])
ks = ks[last:]
names = {"assign": "kmb_assign", "decide": "kmb_seq_strided", "apply": "kmb_seq_apply"}
def kind(n):
    for k, v in names.items():
        if v in n:
            return k
    return None
seq = [(kind(n), s, e, n) for n, s, e in ks]
print("kernels in the last call:", len(seq), "span ms %.2f" % ((seq[-1][2] - seq[0][1]) / 1e6))
tot = {}
for k, s, e, n in seq:
    key = k or n.split("(")[0][:40]
    t = tot.setdefault(key, [0, 0.0])
    t[0] += 1
    t[1] += (e - s) / 1e6
for key, (c, ms) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print("%-42s %6d launches %9.2f ms busy  %7.2f us avg" % (key, c, ms, 1e3 * ms / c))
gaps = [(seq[i + 1][1] - seq[i][2]) / 1e3 for i in range(len(seq) - 1)]
print("sum of gaps between consecutive kernels ms %.2f (median %.2f us, p90 %.2f us)" %
      (sum(gaps) / 1e3, float(np.median(gaps)), float(np.percentile(gaps, 90))))
for a, b in (("assign", "decide"), ("decide", "apply"), ("apply", "assign")):
    g = [(seq[i + 1][1] - seq[i][2]) / 1e3 for i in range(len(seq) - 1) if seq[i][0] == a and seq[i + 1][0] == b]
    if g:
        print("gap %s -> %s: n %d median %.2f us mean %.2f us" % (a, b, len(g), float(np.median(g)), float(np.mean(g))))
for k in names:
    d = [(e - s) / 1e3 for kk, s, e, n in seq if kk == k]
    if d:
        print("%s duration: median %.2f us p10 %.2f p90 %.2f max %.2f" % (k, float(np.median(d)), float(np.percentile(d, 10)),
                                                                        float(np.percentile(d, 90)), max(d)))
