#!/bin/bash
# Round 3: the FProxGD world-2 diagnosis, then the device-control A/B and the C2 A^T R sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_fdc_diag.sh || exit 1
bash scripts/gpu_env_sweep.sh r3_dcab scripts/sweep_dc_r3.txt || exit 1
bash scripts/gpu_env_sweep.sh r3_c2atr scripts/sweep_c2atr.txt || exit 1
echo done
