#!/bin/bash
# Round-3 GPU sessions, one case each (run through gpurun from the repo root):
#   /usr/local/graft/bin/gpurun -- scripts/sessions_r03.sh <letter>
# Each writes gpurun_out/r03<letter>_*.log; the logs kept under profiles/ name their session.
# Steps go through scripts/gpu_session.sh (each under its own time limit; a fault stops the session).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
NB="--no-cpu-baseline --no-count"
W="timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv"
SQA="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P="timeout -s KILL 200 rocprofv3 --output-format csv"
case "$1" in
c)
    # round-3 session C: phase timers (count variant) of C2, C4, C3; the counters rocprofv3 offers on
    # this box; a PC-sampling trial on a C4-shaped render (last: a failure there stops nothing else)
    export TMPDIR=/tmp
    scripts/gpu_session.sh \
      "300:r03c_phases:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16 && python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8 && python scripts/phases.py --scene 5 --width 800 --height 800 --spp 16" \
      "120:r03c_counters:rocprofv3 -L" \
      "180:r03c_pcs:rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 --output-format csv -d gpurun_out/r03c_pcs -o pcs -- python3 bench.py --config C4 --width 960 --height 540 --spp 50 --steps 1 --warmup 0 --no-cpu-baseline --no-count"
    ;;
d)
    # round-3 session D: GPU tests of the relative-BLAS / 16-bit-stack final variant; A/B of the
    # final variant's 16-bit stack (4 waves) vs 32-bit (LDS-bound 3 waves) vs 3-wave registers (C4);
    # rect / box reciprocal divisions (C3, C4, Cornell smoke); phase timers of C4
    scripts/gpu_session.sh tests \
      "500:r03d_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_s32.so $L/librtiow_exp_w3.so $L/librtiow_exp_rectrcp.so $L/librtiow_exp_boxrcp.so --scene 7 --width 1920 --height 1080 --spp 100" \
      "300:r03d_ab_c3:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_rectrcp.so $L/librtiow_exp_boxrcp.so --scene 5 --width 800 --height 800 --spp 200" \
      "300:r03d_ab_c6:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_rectrcp.so $L/librtiow_exp_boxrcp.so --scene 6 --width 600 --height 600 --spp 200" \
      "200:r03d_phases:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
    ;;
e)
    # round-3 session E: C4 A/B of the deferred instance walk and of the final variant's 16-bit stack (4 waves) after the LDS-layout
    # fix, vs the 32-bit stack (LDS-bound 3 waves) and 3-wave registers; C2/C3 of the default build
    scripts/gpu_session.sh \
      "500:r03e_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_s32.so $L/librtiow_exp_nodefer.so --scene 7 --width 1920 --height 1080 --spp 100" \
      "200:r03e_phases:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8" \
      "600:r03e_calib:scripts/calib_r02.sh r03e_calib" \
      bench_c2 bench_c3 tests
    ;;
f)
    # round-3 session F: C4 stack width x register budget (16/32-bit stack entries, 128/168 VGPRs)
    scripts/gpu_session.sh \
      "600:r03f_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_s32.so $L/librtiow_exp_s16w3.so $L/librtiow_exp_s32w3.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 3"
    ;;
g)
    # round-3 session G: GPU tests; C4 A/B of the BLAS top levels staged in LDS; C4 phase timers
    scripts/gpu_session.sh tests \
      "500:r03g_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_nostage.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 3" \
      "200:r03g_phases:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
    ;;
h)
    # round-3 session H: C4 A/B of how many BLAS nodes to stage in LDS (256 = the LDS budget, 64, 16, none)
    scripts/gpu_session.sh \
      "600:r03h_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_b64.so $L/librtiow_exp_b16.so $L/librtiow_exp_nostage.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
    ;;
i)
    # round-3 session I: the committed build end to end — GPU tests, smoke, C1-C5 f64 and C2-C4 f32
    # bench lines, count-variant phase shares (C2, C4 f64, C4 f32)
    PREFIX=r03i_ scripts/gpu_session.sh tests smoke bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4 \
      "200:r03i_phases_c2:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
      "300:r03i_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8" \
      "300:r03i_phases_c4_f32:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8 --precision f32"
    ;;
j)
    # round-3 session J: PMC profiles (kernel trace + SQ/TCC passes) of C2 and C4 at the committed build
    PREFIX=r03j_ scripts/gpu_session.sh prof_c2 prof_c4
    ;;
l)
    # round-3 session L: VALU calibration with the kernel-mix replays (KMIX_C2 / KMIX_C4)
    scripts/gpu_session.sh "600:r03l_calib:scripts/calib_r02.sh r03l_calib"
    ;;
m)
    # round-3 session M: C4 A/B of the shared deferred-walk stack (13 entries instead of 25: 4 blocks per CU)
    scripts/gpu_session.sh \
      "600:r03m_ab_c4:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
      "400:r03m_tests:python -u -m pytest tests/test_gpu_nesting.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread"
    ;;
n)
    # round-3 session N: C4 / C3 / Cornell-smoke A/B: 3-wave build (before the shared stack), the
    # shared stack + normal-derived sphere uv without the stack-address rematerialization, and HEAD
    scripts/gpu_session.sh \
      "600:r03n_ab_c4:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_exp_noremat.so $L/librtiow_amd.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
      "400:r03n_ab_c3:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_exp_noremat.so $L/librtiow_amd.so --scene 5 --width 800 --height 800 --spp 200 --rounds 2" \
      "400:r03n_ab_c6:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_exp_noremat.so $L/librtiow_amd.so --scene 6 --width 600 --height 600 --spp 200 --rounds 2" \
      "600:r03n_tests:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
    ;;
p)
    # round-3 session P: per-sample buffer in tiled order (tiled_record) vs [sample][pixel]: C2 / C4 A/B,
    # the 4-wide TLAS (RT_WIDE) on C2 with its count-variant phases, WRITE_SIZE of C2 and C4 on the new
    # build, GPU tests
    scripts/gpu_session.sh \
      "300:r03p_w4_smoke:RT_LIB_PATH=$PWD/$L/librtiow_exp_w4.so python -c 'import __graft_entry__ as g; g.smoke()'" \
      "400:r03p_ab_c2:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so $L/librtiow_exp_w4.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
      "200:r03p_phases_c2_w4:RT_LIB_PATH=$PWD/$L/librtiow_exp_w4.so python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
      "200:r03p_phases_c2:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
      "600:r03p_ab_c4:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
      "300:r03p_write_c2:export TMPDIR=/tmp; $W -d gpurun_out/r03p_write_c2 -o w -- python3 bench.py --steps 1 --warmup 0 $NB" \
      "300:r03p_write_c4:export TMPDIR=/tmp; $W -d gpurun_out/r03p_write_c4 -o w -- python3 bench.py --config C4 --steps 1 --warmup 0 $NB" \
      tests
    ;;
q)
    # round-3 session Q: WRITE_SIZE calibration on the trace kernel's store width, VALU lane
    # utilisation of the binary and 4-wide (RT_WIDE) C2 walks (1200x800x100), C4 phase shares at HEAD
    scripts/gpu_session.sh \
      "200:r03q_write_calib:export TMPDIR=/tmp; $P --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r03q_write_calib -o w -- scripts/calib/write_calib" \
      "300:r03q_sqa_bin:export TMPDIR=/tmp; $P --pmc $SQA -d gpurun_out/r03q_sqa_bin -o s -- python3 bench.py --steps 2 --warmup 1 --spp 100 $NB" \
      "300:r03q_sqa_w4:export TMPDIR=/tmp RT_LIB_PATH=$PWD/$L/librtiow_exp_w4.so; $P --pmc $SQA -d gpurun_out/r03q_sqa_w4 -o s -- python3 bench.py --steps 2 --warmup 1 --spp 100 $NB" \
      "300:r03q_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
    ;;
r)
    # round-3 session R: final-scene variant in 512-thread workgroups (one LDS copy of the TLAS per
    # 8 waves: RT_BLOCK_FINAL=512), with the BLAS staging cap at 64 nodes and lifted; GPU tests
    scripts/gpu_session.sh \
      "600:r03r_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_b512.so $L/librtiow_exp_b512all.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
      tests
    ;;
s)
    # round-3 session S: the committed build end to end — GPU tests, smoke, bench lines C1-C5 (f64) and
    # C2-C4 (f32), PMC profiles of C2 / C3 / C4 (the roofline bench.py quotes for this source hash),
    # C4 phase shares
    PREFIX=r03s_ scripts/gpu_session.sh tests smoke bench bench_c4 prof_c2 prof_c4 bench_c1 bench_c3 bench_c5 prof_c3 f32_c2 f32_c3 f32_c4 \
      "300:r03s_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
    ;;
t)
    # round-3 session T: the final variant with per-ray reciprocals of the direction for its rect / box
    # tests (RT_RECT_RCP_FINAL; 127 VGPRs, no spills at 4 waves) vs the committed build (r03s) and the
    # instance rays' set-up restricted to their child's features; C4 and C3
    scripts/gpu_session.sh \
      "600:r03t_ab_c4:python scripts/ab_builds.py $L/librtiow_exp_r03s.so $L/librtiow_amd.so $L/librtiow_exp_rcpf.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
      "400:r03t_ab_c3:python scripts/ab_builds.py $L/librtiow_exp_r03s.so $L/librtiow_amd.so --scene 5 --width 800 --height 800 --spp 200 --rounds 2"
    ;;
u)
    # round-3 session U: rank 0's row shard of C2 for N = 1, 2, 4, 8 on one GPU (the multi-GPU
    # scaling loss from tile coherence, apart from the gather), rows and 8-row bands
    scripts/gpu_session.sh "400:r03u_shard:python scripts/shard_coherence.py --spp 500 --reps 3"
    ;;
v)
    # round-3 session V: rank 0's row shard of C2 for 2-, 4- and 8-row bands (N = 2, 4, 8)
    scripts/gpu_session.sh "400:r03v_shard:python scripts/shard_coherence.py --spp 500 --reps 3 --row-blocks 2 4 8"
    ;;
w)
    # round-3 session W: tile shards (rt_render_params.tile_shard) — rank 0's C2 shard at N = 2, 4, 8
    # against row shards; GPU tests (tile-shard reassembly, bench.py N = 2 tiles / N = 3 rows)
    scripts/gpu_session.sh "400:r03w_shard:python scripts/shard_coherence.py --spp 500 --reps 3 --row-blocks 1 --tiles" \
      "900:r03w_gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread"
    ;;
x)
    # round-3 session X: the final build end to end — smoke, bench lines (C2 default, C4), PMC profiles
    # of C2 and C4 at this source hash (the roofline bench.py quotes)
    PREFIX=r03x_ scripts/gpu_session.sh smoke bench bench_c4 prof_c2 prof_c4
    ;;
y)
    # round-3 session Y: the final variant testing the huge root-child leaf (the r = 5000 fog medium)
    # before its walk with the whole wave (RT_PRELEAF_FINAL; 126 VGPRs, 6 spilled) vs HEAD, C4
    scripts/gpu_session.sh \
      "600:r03y_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_prefinal.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
    ;;
z)
    # round-3 session Z: session Y's A/B (librtiow_exp_prefinal.so built with -DRT_PRELEAF_FINAL=1 on
    # the flag's definition, not kept in the tree) then session X (smoke, bench lines, PMC at HEAD)
    scripts/gpu_session.sh \
      "600:r03z_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_prefinal.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" && \
    PREFIX=r03x_ scripts/gpu_session.sh smoke bench bench_c4 prof_c2 prof_c4
    ;;
final)
    # round-3 closing check of HEAD as the driver runs it (GPU tests, smoke, bench.py with no
    # arguments), C4's bench line, and the PMC passes of C2 / C4 at this source hash
    PREFIX=r03_final_ scripts/gpu_session.sh tests smoke bench bench_c4 prof_c2 prof_c4
    ;;
final2)
    # the remaining bench lines at HEAD's source hash: C1, C3, C5 (f64), C2-C4 (f32), C3's PMC passes
    PREFIX=r03_final_ scripts/gpu_session.sh bench_c1 bench_c3 bench_c5 f32_c2 f32_c3 f32_c4 prof_c3
    ;;
probe)
    # timing probes (NOT the product; built from a copy of csrc with RT_PROBE_NO_NOISE /
    # RT_PROBE_NO_IMAGE: the noise / image texture returns a constant; paths unchanged): the share
    # of the final scene's time its Perlin and image textures take, C4 1920x1080x100
    scripts/gpu_session.sh \
      "700:r03_probe_tex_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_probe_nonoise.so $L/librtiow_probe_noimage.so $L/librtiow_probe_notex.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
    ;;
*) echo "usage: scripts/sessions_r03.sh <session letter>" >&2; exit 2 ;;
esac
