"""Per-kernel times from rocprofv3 --kernel-trace runs (the default rocpd sqlite output):
for each run directory, the kernels of the last 300 frames grouped by name and grid, with
average duration and time per frame.  Usage: python scripts/kernel_times_db.py DIR [DIR ...]"""
import sqlite3, sys, glob, re
def short(n):
    m = re.search(r'(first_bounce_kernel|wf_bounce_kernel|wf_seg_scan_kernel|wf_compact_sort_kernel|wf_local_sort_kernel|copyBuffer|fill\w*)', n)
    return m.group(1) if m else n[:30]
for d in sys.argv[1:]:
    db = glob.glob(f"{d}/**/*.db", recursive=True)[0]
    con = sqlite3.connect(db)
    rows = list(con.execute("select name, start, end, grid_x from kernels order by start"))
    # timed region: last 300 frames -> take kernels after the last 'first_bounce' minus 300
    fb = [i for i, r in enumerate(rows) if 'first_bounce' in r[0]]
    lo = fb[-300]
    sel = rows[lo:]
    agg = {}
    for n, s, e, g in sel:
        k = short(n)
        a = agg.setdefault((k, g), [0, 0.0])
        a[0] += 1; a[1] += (e - s) / 1000.0
    span = (sel[-1][2] - sel[0][1]) / 1000.0 / 300
    print("==", d, "frame span us %.1f" % span)
    busy = 0
    for (k, g), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print("  %-24s grid %-8d calls %5d avg %8.1f us  per-frame %8.1f" % (k, g, c, t / c, t / 300))
        busy += t / 300
    print("  kernel sum per frame %.1f, gaps %.1f" % (busy, span - busy))
