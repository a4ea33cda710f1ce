#!/bin/bash
# folded lip Conv3d forward for the Cin = 1 front-ends: avse4 C4 (16, 1, 125, 112, 112) probe with a find pass
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -rf gpurun_out/miopen_db && cp -r avse_challenge_amd/miopen_db gpurun_out/miopen_db
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 500 python tools/conv3d_fold_probe.py 16,1,125,112,112 > gpurun_out/fold_probe_a4.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/fold_probe_a4.log | tail -4; exit $rc
