#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy of trace_kernel.hip (compiler remarks), compact.

usage: [RT_VARIANT_SRC=trace_v_spheres.hip] python scripts/res_usage.py [-DRT_TRACE_LOOP=2 ...]   (extra hipcc flags)
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.environ.get("RT_CSRC", os.path.join(REPO, "rust-ray-tracing-in-a-weekend_amd", "csrc"))
src = os.path.join(CSRC, os.environ.get("RT_VARIANT_SRC", "trace_v_all.hip"))
sys.path.insert(0, REPO)
import __graft_entry__ as ge  # noqa: E402  (the library's own flags)
cmd = ["/opt/rocm/bin/hipcc", *[f for f in ge.CXXFLAGS if f not in ("-Wall", "-Wno-unused-function")],
       "--cuda-device-only", "-c", src, "-o", "/tmp/res_usage.o", "-Rpass-analysis=kernel-resource-usage", *sys.argv[1:]]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(.+?): (\d+) \[", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    n = r["name"]
    m = re.search(r"(trace_chunks|trace_pool)INS_3CfgILj(\d+)ELb(\d)ELb(\d)ELb(\d)ELb(\d)E(?:Lb(\d)E)?EE(?:Lb(\d)E)?", n)
    if not m:
        continue
    kern, f, s32, lds, nall, count, f32, items = m.groups()
    if items == "1":
        kern = "trace_items"
    if count == "1":
        continue
    print(f"{kern:12s} F={f:>2}{' f32' if f32 == '1' else ''} s32={s32} lds={lds} nall={nall}: VGPRs {r.get('VGPRs')} AGPRs {r.get('AGPRs')} "
          f"SGPRs {r.get('TotalSGPRs')} spills {r.get('VGPRs Spill')}/{r.get('SGPRs Spill')} scratch {r.get('ScratchSize [bytes/lane]', r.get('ScratchSize'))} "
          f"occupancy {r.get('Occupancy [waves/SIMD]', r.get('Occupancy'))} LDS {r.get('LDS Size [bytes/block]')}")
