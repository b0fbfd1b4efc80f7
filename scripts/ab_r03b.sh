#!/bin/bash
# round-3 session B: VALU calibration of v_pk_fma_f32 / max3 / med3; A/B of machine LICM, the
# final-scene variant's waves, rolled Perlin loops and the op_sel packed slab FMA (C2, C4, C3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh \
  "120:r03b_calib:scripts/calib/valu_calib pk_fma_f32,f32_fma,max3_f32,med3_f32,min_f32,f32_add sat,one 4000" \
  "400:r03b_ab_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_old.so $L/librtiow_exp_licm.so $L/librtiow_exp_pk.so --scene 0 --width 1200 --height 800 --spp 500" \
  "500:r03b_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_old.so $L/librtiow_exp_licm.so $L/librtiow_exp_w3.so $L/librtiow_exp_unroll.so $L/librtiow_exp_pk.so --scene 7 --width 1920 --height 1080 --spp 100" \
  "300:r03b_ab_c3:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_old.so $L/librtiow_exp_pk.so --scene 5 --width 800 --height 800 --spp 200" \
  tests
