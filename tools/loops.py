#!/usr/bin/env python3
"""List the loops (backward branches) of one kernel in a device .s file with instruction mix."""
import re
import sys

path, kern = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "_ZN4d2dk15d2d_step_kernelILb1EEEvNS_8StepArgsE")
t = open(path).read()
t = t[t.index(kern + ":"):]
t = t[: t.index(".Lfunc_end")]
L = t.split("\n")
labels = {m.group(1): i for i, l in enumerate(L) if (m := re.match(r"^(\.LBB\w+):", l))}
for i, l in enumerate(L):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    if tgt in labels and labels[tgt] < i:
        body = [x.strip() for x in L[labels[tgt]:i]]
        ins = [x for x in body if x and not x.startswith((".", ";")) and not x.endswith(":")]
        cnt = lambda pat: sum(1 for x in ins if re.search(pat, x))
        if len(ins) > int(sys.argv[3] if len(sys.argv) > 3 else 30):
            print(f"loop {tgt:10s} lines {labels[tgt]}-{i} instrs {len(ins)} f64 {cnt('_f64')} "
                  f"ds {cnt('^ds_')} scratch {cnt('scratch_')} saveexec {cnt('saveexec')} salu {cnt('^s_')}")
