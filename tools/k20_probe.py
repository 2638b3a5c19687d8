"""Per-launch K1 durations of the 20/5 bench runs traced by tools/k20_probe.sh.

For each traced run: the bench line's value, then every d2d_step_kernel launch in order (us), the
mean of the last 20 (the timed region) and the gaps between their starts.
Usage: python tools/k20_probe.py gpurun_out/k20_TAG
"""
import csv
import glob
import json
import os
import sys


def line(path):
    try:
        with open(path) as f:
            return json.loads(f.read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        return None


def main(out):
    for p in sorted(glob.glob(os.path.join(out, "plain_*.log"))):
        d = line(p)
        if d:
            print(f"{os.path.basename(p)}: {d['value'] / 1e9:.3f} G  ms/step {d['ms_per_step'] * 1e3:.2f} us"
                  f"  K1 {d['roofline']['kernel_ms'] * 1e3:.2f} us")
    for kdir in sorted(glob.glob(os.path.join(out, "kt_*"))):
        if not os.path.isdir(kdir):
            continue
        d = line(kdir + ".log")
        csvs = glob.glob(os.path.join(kdir, "**", "*kernel_trace.csv"), recursive=True)
        if not csvs:
            continue
        rows = []
        with open(csvs[0]) as f:
            for r in csv.DictReader(f):
                if "d2d_step_kernel" in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        rows.sort()
        dur = [(e - s) / 1e3 for s, e in rows]
        timed = rows[-20:]
        tdur = dur[-20:]
        gaps = [(timed[i + 1][0] - timed[i][1]) / 1e3 for i in range(len(timed) - 1)]
        head = f"{os.path.basename(kdir)}: " + (f"{d['value'] / 1e9:.3f} G" if d else "no line")
        print(f"{head}  launches {len(dur)}  timed mean {sum(tdur) / len(tdur):.2f} us"
              f"  min {min(tdur):.2f}  max {max(tdur):.2f}  mean gap {sum(gaps) / max(len(gaps), 1):.2f} us")
        print("  all K1 (us):", " ".join(f"{x:.1f}" for x in dur))


if __name__ == "__main__":
    main(sys.argv[1])
