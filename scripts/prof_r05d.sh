set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
A="--spp 16 --reps 1 --paths 0"
timeout -k 10 200 python3 -u scripts/wf_sweep.py $A --count > $O/sweep.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/pa -o pa -- python3 scripts/wf_sweep.py $A > $O/pa.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $O/pb -o pb -- python3 scripts/wf_sweep.py $A > $O/pb.log 2>&1 || exit 5
ls $O/pa $O/pb
