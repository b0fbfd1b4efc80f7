#!/bin/bash
# Kernel trace + SQ wait counters of the wavefront A/B (scripts/wf_sweep.py) on the GPU box.
# usage: scripts/prof_wf.sh TAG "<wf_sweep args>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
A=${2:-"--spp 16 --reps 1 --paths 0"}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 scripts/wf_sweep.py $A > $O/kt.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/pa -o pa -- python3 scripts/wf_sweep.py $A > $O/pa.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --output-format csv -d $O/pb -o pb -- python3 scripts/wf_sweep.py $A > $O/pb.log 2>&1 || exit 5
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o pf -- python3 scripts/wf_sweep.py $A > $O/pf.log 2>&1 || exit 6
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o pw -- python3 scripts/wf_sweep.py $A > $O/pw.log 2>&1 || exit 7
python3 - "$O" <<'PY'
import csv, collections, sys
o = sys.argv[1]
for r in csv.DictReader(open(f"{o}/kt/kt_kernel_stats.csv")):
    print("kt", r["Name"][:48], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3), "total_ms %.2f" % (float(r["TotalDurationNs"]) / 1e6))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for t in ("pa", "pb", "pf", "pw"):
    for r in csv.DictReader(open(f"{o}/{t}/{t}_counter_collection.csv")):
        agg[r["Kernel_Name"][:48]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if v.get("SQ_WAVE_CYCLES", 0) > 1e8:
        print("pmc", k, "wait/wave %.3f" % (v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"]),
              "lane_util %.3f" % (v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_INSTS_VALU"])),
              "dram_GB %.2f" % ((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) / 1e6), {c: "%.3e" % x for c, x in v.items()})
PY
