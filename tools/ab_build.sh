#!/usr/bin/env bash
# Diagnostic A/B timing builds (not parity builds): libhandarm_hip_<name>.so with -DHA_AB_TIMING and one phase
# repeated, so (time with the phase twice) - (product time) = the phase's cost in the real schedule.
# Usage: bash tools/ab_build.sh NAME "-DFLAG ..."   (run here, on the CPU; the .so travels to the GPU box)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result \
  -I "$R/include" -DHA_AB_TIMING "$@" -o "$R/isaacgym-hand-arm_amd/handarm_hip/libhandarm_hip_$NAME.so" \
  "$R/isaacgym-hand-arm_amd/csrc/handarm_hip.hip"
