#!/bin/bash
# Round-4 GPU sessions, one case each (run through gpurun from the repo root):
#   /usr/local/graft/bin/gpurun -- scripts/sessions_r04.sh <letter>
# Each writes gpurun_out/r04<letter>_*.log; the logs kept under profiles/ name their session.
# Steps go through scripts/gpu_session.sh (each under its own time limit; a fault stops the session).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
NB="--no-cpu-baseline --no-count"
case "$1" in
a)
    # round-4 session A: the byte-exact output / RCCL-branch / empty-shard build — GPU tests, smoke, default bench
    PREFIX=r04a_ scripts/gpu_session.sh tests smoke bench
    ;;
b)
    # round-4 session B: GPU tests with the Box candidate-side test; A/B of the rejection-loop cap
    # (RT_TRY_LEFT 2/4/8, RT_TRY_MIN 1) on C2 and of the candidate sides on C4; phase timers of
    # C4 (candidates) and of C2 under the cap
    scripts/gpu_session.sh tests \
      "600:r04b_ab_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_try2.so $L/librtiow_exp_try4.so $L/librtiow_exp_try8.so $L/librtiow_exp_try4m1.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
      "600:r04b_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_nocand.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 3" \
      "200:r04b_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8" \
      "200:r04b_phases_c4_nocand:RT_LIB_PATH=$L/librtiow_exp_nocand.so python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8" \
      "200:r04b_phases_c2:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
      "200:r04b_phases_c2_try4:RT_LIB_PATH=$L/librtiow_exp_try4.so python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16"
    ;;
c)
    # round-4 session C: GPU tests (RT_TRY_LEFT 4 default, box candidates off); A/B of walk suspension
    # (RT_PAUSE 4/8/16/32) and of the rejection cap off on C2; the cap on C4; phase timers under suspension
    scripts/gpu_session.sh tests \
      "600:r04c_ab_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_try0.so $L/librtiow_exp_pause4.so $L/librtiow_exp_pause8.so $L/librtiow_exp_pause16.so $L/librtiow_exp_pause32.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
      "600:r04c_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_try0.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 3" \
      "200:r04c_phases_c2:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
      "200:r04c_phases_c2_pause8:RT_LIB_PATH=$L/librtiow_exp_pause8.so python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
      "200:r04c_phases_c2_pause16:RT_LIB_PATH=$L/librtiow_exp_pause16.so python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16"
    ;;
d)
    # round-4 session D: walk suspension refined (a resumed walk is not suspended again; later
    # first suspension) on C2; the rejection cap on every variant (RT_TRY_ALL) on C3 / C4; VALU lane
    # counters (SQ pass) of the default build and of the best suspension build on C2; GPU tests
    export TMPDIR=/tmp
    SQA="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
    B="--steps 2 --warmup 1 --no-cpu-baseline --no-count"
    scripts/gpu_session.sh \
      "600:r04d_ab_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_p8once.so $L/librtiow_exp_p8once_m5.so $L/librtiow_exp_p16once.so $L/librtiow_exp_p8m6.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
      "600:r04d_ab_c3:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_tryall.so --scene 5 --width 800 --height 800 --spp 200 --rounds 3" \
      "600:r04d_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_tryall.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
      "200:r04d_phases_c2_p8once:RT_LIB_PATH=$L/librtiow_exp_p8once.so python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
      "300:r04d_sqa_default:timeout -s KILL 240 rocprofv3 --pmc $SQA --output-format csv -d gpurun_out/r04d_sqa_default -o sqa -- python3 bench.py $B" \
      "300:r04d_sqa_p8once:RT_LIB_PATH=$L/librtiow_exp_p8once.so timeout -s KILL 240 rocprofv3 --pmc $SQA --output-format csv -d gpurun_out/r04d_sqa_p8once -o sqa -- python3 bench.py $B" \
      "300:r04d_sqa_pause8:RT_LIB_PATH=$L/librtiow_exp_p8m6.so timeout -s KILL 240 rocprofv3 --pmc $SQA --output-format csv -d gpurun_out/r04d_sqa_p8m6 -o sqa -- python3 bench.py $B" \
      tests
    ;;
e)
    # round-4 session E: the bounded trace-output buffer (4 GB default, overlapped batches) — GPU tests;
    # C2 and C4 bench lines at the default bound, at a 128 GB bound (one batch, round 3's behaviour)
    # and at 4 GB without overlap (batches in order)
    NB="--no-cpu-baseline --no-count"
    scripts/gpu_session.sh tests \
      "300:r04e_c2_bound4g:python bench.py --steps 10 --warmup 2 $NB" \
      "300:r04e_c2_onebatch:RT_SAMPLE_BUF_MB=131072 python bench.py --steps 10 --warmup 2 $NB" \
      "300:r04e_c2_serial:RT_BATCH_OVERLAP=0 python bench.py --steps 10 --warmup 2 $NB" \
      "300:r04e_c2_bound4g_b:python bench.py --steps 10 --warmup 2 $NB" \
      "400:r04e_c4_bound4g:python bench.py --config C4 --steps 3 --warmup 1 $NB" \
      "400:r04e_c4_onebatch:RT_SAMPLE_BUF_MB=131072 python bench.py --config C4 --steps 3 --warmup 1 $NB" \
      "400:r04e_c4_serial:RT_BATCH_OVERLAP=0 python bench.py --config C4 --steps 3 --warmup 1 $NB"
    ;;
f)
    # round-4 session F: the item pool under the 4 GB bound (C4: its partials fit one batch) against
    # the per-sample pool in one batch; C2 items; C5 at the bound (items, overlapped batches) vs one batch
    NB="--no-cpu-baseline --no-count"
    scripts/gpu_session.sh \
      "400:r04f_c4_items:RT_SCHEDULE=2 python bench.py --config C4 --steps 3 --warmup 1 $NB" \
      "400:r04f_c4_items_blk4:RT_SCHEDULE=2 RT_BLOCK_CHUNKS=4 python bench.py --config C4 --steps 3 --warmup 1 $NB" \
      "400:r04f_c4_onebatch:RT_SAMPLE_BUF_MB=131072 python bench.py --config C4 --steps 3 --warmup 1 $NB" \
      "300:r04f_c2_items:RT_SCHEDULE=2 python bench.py --steps 10 --warmup 2 $NB" \
      "300:r04f_c2_default:python bench.py --steps 10 --warmup 2 $NB" \
      "600:r04f_c5_default:python bench.py --config C5 --steps 1 --warmup 1 $NB" \
      "600:r04f_c5_onebatch:RT_SAMPLE_BUF_MB=131072 python bench.py --config C5 --steps 1 --warmup 1 $NB"
    ;;
g)
    # round-4 session G (final build): GPU tests, smoke, rocprofv3 kernel trace + PMC passes of C1-C5
    PREFIX=r04g_ scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 prof_c4
    ;;
g2)
    PREFIX=r04g_ scripts/gpu_session.sh prof_c5
    ;;
h)
    # round-4 session H: VALU calibration incl. the kmix replays of C2 / C3 / C4 (gen_kmix.py on r04g's PMC)
    scripts/gpu_session.sh "600:r04h_calib:scripts/calib_r02.sh r04h_calib"
    ;;
i)
    # round-4 session I: the final bench lines (roofline from r04g's PMC and r04h's calibration), C1-C5 f64,
    # the default bench line the driver runs, f32 lines of C2-C4
    PREFIX=r04i_ scripts/gpu_session.sh bench bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4
    ;;
j)
    # round-4 session J: walk suspension with the parked state in LDS (12 B per lane after the stack; built
    # from a copy of csrc, scripts/sessions_r04.sh j) against the default on C2; phases and SQ pass of K = 8
    export TMPDIR=/tmp
    SQA="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
    B="--steps 2 --warmup 1 --no-cpu-baseline --no-count"
    scripts/gpu_session.sh \
      "600:r04j_ab_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_ldsp8.so $L/librtiow_exp_ldsp8once.so $L/librtiow_exp_ldsp16once.so $L/librtiow_exp_ldsp4.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
      "200:r04j_phases_c2_ldsp8:RT_LIB_PATH=$L/librtiow_exp_ldsp8.so python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
      "300:r04j_sqa_ldsp8:RT_LIB_PATH=$L/librtiow_exp_ldsp8.so timeout -s KILL 240 rocprofv3 --pmc $SQA --output-format csv -d gpurun_out/r04j_sqa_ldsp8 -o sqa -- python3 bench.py $B"
    ;;
jg)
    # sessions J and G in one call (boxes are scarce): the LDS suspension A/B, then the final-build passes
    "$0" j && "$0" g
    ;;
k)
    # round-4 session K: the final scene's instanced cluster dissolved into the top-level tree
    # (RT_INST_DISSOLVE=1, flatten.cpp) — nesting tests incl. bit identity with the nested walk; A/B on C4
    # against the deferred BLAS walk; phase timers of C4 dissolved
    scripts/gpu_session.sh \
      "400:r04k_gpu_tests_nesting:python -u -m pytest tests/test_gpu_nesting.py -x -v --timeout 120 --timeout-method thread" \
      "600:r04k_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_amd.so@RT_INST_DISSOLVE=1 $L/librtiow_amd.so@RT_INST_DISSOLVE=1,RT_DISSOLVE_CI=0.35 $L/librtiow_amd.so@RT_INST_DISSOLVE=1,RT_DISSOLVE_CI=0.25 --scene 7 --width 1920 --height 1080 --spp 100 --rounds 3" \
      "200:r04k_phases_c4_dissolve:RT_INST_DISSOLVE=1 RT_DISSOLVE_CI=0.35 python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8" \
      "200:r04k_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
    ;;
k2)
    # round-4 session K2: the single-primitive instance rays without node-slab set-up (and the BVH-only
    # deferral) against the build before it (librtiow_exp_prev.so, commit 7d4bc81) on C3 and C4
    scripts/gpu_session.sh \
      "600:r04k2_ab_c3:python scripts/ab_builds.py $L/librtiow_exp_prev.so $L/librtiow_amd.so --scene 5 --width 800 --height 800 --spp 200 --rounds 3" \
      "600:r04k2_ab_c4:python scripts/ab_builds.py $L/librtiow_exp_prev.so $L/librtiow_amd.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
    ;;
kk)
    # sessions K and K2 in one call
    "$0" k && "$0" k2
    ;;
m)
    # round-4 session M (final build, after K): GPU tests, smoke, rocprofv3 kernel trace + PMC passes of C1-C4
    PREFIX=r04m_ scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 prof_c4
    ;;
m2)
    # session M2: C5's passes, then the VALU calibration with the kmix replays of M's PMC (gen_kmix.py)
    PREFIX=r04m_ scripts/gpu_session.sh prof_c5 && scripts/gpu_session.sh "600:r04m_calib:scripts/calib_r02.sh r04m_calib"
    ;;
n)
    # session N: the final bench lines (roofline from M's PMC and M2's calibration), C1-C5 f64, the
    # default line the driver runs, f32 lines of C2-C4
    PREFIX=r04n_ scripts/gpu_session.sh bench bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4
    ;;
q)
    # session Q: one-leaf top levels (Cornell scenes) walked as a wave-uniform slot loop (scalar records and
    # kind dispatch; librtiow_exp_uleaf.so, built from a csrc copy with RT_UNIFORM_LEAF) against HEAD on C3
    # and Cornell smoke; C3's phase timers at HEAD
    scripts/gpu_session.sh \
      "600:r04q_ab_c3:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_uleaf.so --scene 5 --width 800 --height 800 --spp 200 --rounds 3" \
      "600:r04q_ab_smoke:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_uleaf.so --scene 6 --width 800 --height 800 --spp 200 --rounds 3" \
      "200:r04q_phases_c3:python scripts/phases.py --scene 5 --width 800 --height 800 --spp 16"
    ;;
r)
    # session R: the uniform one-leaf walk (uleaf), + wave-uniform kind / instance index (uleaf2), + one finisher
    # for top-level and instanced primitives and for rects / box sides (uleaf3), each from a csrc copy, against
    # HEAD on C3 and Cornell smoke; uleaf3 on C4 (its box-side finisher change)
    E="$L/librtiow_exp_uleaf.so $L/librtiow_exp_uleaf2.so $L/librtiow_exp_uleaf3.so"
    scripts/gpu_session.sh \
      "600:r04r_ab_c3:python scripts/ab_builds.py $L/librtiow_amd.so $E --scene 5 --width 800 --height 800 --spp 200 --rounds 3" \
      "600:r04r_ab_smoke:python scripts/ab_builds.py $L/librtiow_amd.so $E --scene 6 --width 800 --height 800 --spp 200 --rounds 3" \
      "600:r04r_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_uleaf3.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
    ;;
s)
    # round-4 session S (final build, after the one-leaf loop): GPU tests, smoke, PMC passes of C1-C4
    PREFIX=r04s_ scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 prof_c4
    ;;
s2)
    # session S2: C5's passes, then the VALU calibration with the kmix replays of S's PMC
    PREFIX=r04s_ scripts/gpu_session.sh prof_c5 && scripts/gpu_session.sh "600:r04s_calib:scripts/calib_r02.sh r04s_calib"
    ;;
t)
    # session T: the final bench lines of this build (C1-C5 f64, the default line, f32 C2-C4)
    PREFIX=r04t_ scripts/gpu_session.sh bench bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4
    ;;
st)
    # sessions S and T in one call (boxes are scarce): tests, smoke, PMC passes of C1-C5, their pmc.json
    # entries written on the box (scripts/pmc_r02.py, the same step the builder runs after merging), then
    # the bench lines, which read them
    PREFIX=r04s_ scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 prof_c4 prof_c5 && \
    python scripts/pmc_r02.py bench r04s_prof_c1 r04_final_c1 0,1200,800,10,8,1,1 "round-4 final build (r04s)" && \
    python scripts/pmc_r02.py bench r04s_prof_c2 r04_final_c2 0,1200,800,500,50,1,1 "round-4 final build (r04s)" && \
    python scripts/pmc_r02.py bench r04s_prof_c3 r04_final_c3 5,800,800,1000,50,1,1 "round-4 final build (r04s)" && \
    python scripts/pmc_r02.py bench r04s_prof_c4 r04_final_c4 7,1920,1080,1000,50,1,1 "round-4 final build (r04s)" && \
    python scripts/pmc_r02.py bench r04s_prof_c5 r04_final_c5 0,4096,4096,4096,50,1,2 "round-4 final build (r04s)" && \
    "$0" t
    ;;
st2)
    # ST for the box-pairs build (prefixes r04x_ / r04y_): sessions S and T in one call (boxes are scarce): tests, smoke, PMC passes of C1-C5, their pmc.json
    # entries written on the box (scripts/pmc_r02.py, the same step the builder runs after merging), then
    # the bench lines, which read them
    PREFIX=r04x_ scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 prof_c4 prof_c5 && \
    python scripts/pmc_r02.py bench r04x_prof_c1 r04_final_c1 0,1200,800,10,8,1,1 "round-4 final build (r04x)" && \
    python scripts/pmc_r02.py bench r04x_prof_c2 r04_final_c2 0,1200,800,500,50,1,1 "round-4 final build (r04x)" && \
    python scripts/pmc_r02.py bench r04x_prof_c3 r04_final_c3 5,800,800,1000,50,1,1 "round-4 final build (r04x)" && \
    python scripts/pmc_r02.py bench r04x_prof_c4 r04_final_c4 7,1920,1080,1000,50,1,1 "round-4 final build (r04x)" && \
    python scripts/pmc_r02.py bench r04x_prof_c5 r04_final_c5 0,4096,4096,4096,50,1,2 "round-4 final build (r04x)" && \
    PREFIX=r04y_ scripts/gpu_session.sh bench bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4
    ;;
st3)
    # ST for the box-pairs build (prefixes r04z_ / r04y_): sessions S and T in one call (boxes are scarce): tests, smoke, PMC passes of C1-C5, their pmc.json
    # entries written on the box (scripts/pmc_r02.py, the same step the builder runs after merging), then
    # the bench lines, which read them
    PREFIX=r04z_ scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 prof_c4 prof_c5 && \
    python scripts/pmc_r02.py bench r04z_prof_c1 r04_final_c1 0,1200,800,10,8,1,1 "round-4 final build (r04z)" && \
    python scripts/pmc_r02.py bench r04z_prof_c2 r04_final_c2 0,1200,800,500,50,1,1 "round-4 final build (r04z)" && \
    python scripts/pmc_r02.py bench r04z_prof_c3 r04_final_c3 5,800,800,1000,50,1,1 "round-4 final build (r04z)" && \
    python scripts/pmc_r02.py bench r04z_prof_c4 r04_final_c4 7,1920,1080,1000,50,1,1 "round-4 final build (r04z)" && \
    python scripts/pmc_r02.py bench r04z_prof_c5 r04_final_c5 0,4096,4096,4096,50,1,2 "round-4 final build (r04z)" && \
    PREFIX=r04zb_ scripts/gpu_session.sh bench bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4
    ;;
st4)
    # ST for the box-pairs build (prefixes r04v2_ / r04y_): sessions S and T in one call (boxes are scarce): tests, smoke, PMC passes of C1-C5, their pmc.json
    # entries written on the box (scripts/pmc_r02.py, the same step the builder runs after merging), then
    # the bench lines, which read them
    PREFIX=r04v2_ scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 prof_c4 prof_c5 && \
    python scripts/pmc_r02.py bench r04v2_prof_c1 r04_final_c1 0,1200,800,10,8,1,1 "round-4 final build (r04v2)" && \
    python scripts/pmc_r02.py bench r04v2_prof_c2 r04_final_c2 0,1200,800,500,50,1,1 "round-4 final build (r04v2)" && \
    python scripts/pmc_r02.py bench r04v2_prof_c3 r04_final_c3 5,800,800,1000,50,1,1 "round-4 final build (r04v2)" && \
    python scripts/pmc_r02.py bench r04v2_prof_c4 r04_final_c4 7,1920,1080,1000,50,1,1 "round-4 final build (r04v2)" && \
    python scripts/pmc_r02.py bench r04v2_prof_c5 r04_final_c5 0,4096,4096,4096,50,1,2 "round-4 final build (r04v2)" && \
    PREFIX=r04vb_ scripts/gpu_session.sh bench bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4
    ;;
w3)
    # session W3: pairs holding a Box, a medium or an instance over a BVH split (heavy pairs) against the
    # BLAS-pairs build's rule (only Boxes; RT_BVH_BOXPAIRS=0 turns both off) and every pair split, on C4
    A=$L/librtiow_amd.so
    scripts/gpu_session.sh \
      "600:r04w3_ab_c4:python scripts/ab_builds.py $A $A@RT_BVH_BOXPAIRS=0 $A@RT_BVH_LEAFN=1 --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
    ;;
stw3)
    "$0" w3 && "$0" st4
    ;;
w2)
    # session W2: pairs split inside BLASes too (split_blas_pairs) against the box-pairs build
    # (RT_BVH_BLASPAIRS=0) and every pair split (RT_BVH_LEAFN=1) on C4
    A=$L/librtiow_amd.so
    scripts/gpu_session.sh \
      "600:r04w2_ab_c4:python scripts/ab_builds.py $A $A@RT_BVH_BLASPAIRS=0 $A@RT_BVH_LEAFN=1 --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
    ;;
stw2)
    "$0" w2 && "$0" st3
    ;;
u)
    # session U: the VALU calibration with the kmix replays of the final build's mixes (C3's changed with the
    # one-leaf loop), then C3's and the default bench lines priced by it
    scripts/gpu_session.sh "600:r04u_calib:scripts/calib_r02.sh r04u_calib"
    ;;
u2)
    PREFIX=r04u_ scripts/gpu_session.sh bench bench_c2 bench_c3 bench_c4
    ;;
uu)
    # U, its calibration block written on the box (scripts/pmc_r02.py calib), then the default, C2, C3 and C4 lines
    "$0" u && python scripts/pmc_r02.py calib r04u_calib r04u && "$0" u2
    ;;
v)
    # session V: the SAH build parameters re-swept at HEAD (host-side env, same library): C4 and C2
    A=$L/librtiow_amd.so
    scripts/gpu_session.sh \
      "600:r04v_ab_c4:python scripts/ab_builds.py $A $A@RT_BVH_CI=0.7 $A@RT_BVH_CI=0.85 $A@RT_BVH_LEAFN=1 $A@RT_BVH_CI=0.7,RT_BVH_LEAFN=1 --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
      "600:r04v_ab_c2:python scripts/ab_builds.py $A $A@RT_BVH_CI=0.7 $A@RT_BVH_CI=0.85 --scene 0 --width 1200 --height 800 --spp 100 --rounds 3"
    ;;
w)
    # session W: Box pairs split by the SAH (flatten.cpp split_box_pairs) against the old rule and against
    # every pair split (RT_BVH_LEAFN=1) on C4, same library
    A=$L/librtiow_amd.so
    scripts/gpu_session.sh \
      "600:r04w_ab_c4:python scripts/ab_builds.py $A $A@RT_BVH_BOXPAIRS=0 $A@RT_BVH_LEAFN=1 --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
    ;;
stw)
    # W, then the final-build passes and lines (ST) of this build
    "$0" w && "$0" st2
    ;;
ph)
    # session PH: phase timers of HEAD's build on C4, C3 and C2 (count variants)
    scripts/gpu_session.sh \
      "200:r04ph_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8" \
      "200:r04ph_phases_c3:python scripts/phases.py --scene 5 --width 800 --height 800 --spp 16" \
      "200:r04ph_phases_c2:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16"
    ;;
g2h)
    # sessions G2 (C5's passes) and H (calibration with the r04 kmix replays) in one call
    "$0" g2 && "$0" h
    ;;
*)
    echo "unknown session: $1" >&2; exit 2 ;;
esac
