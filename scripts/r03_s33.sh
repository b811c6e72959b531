#!/bin/bash
# Instruction mix by part of the final round-3 build (diagnostic build, scripts/r03_s15.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S15_OUT=s33 bash scripts/r03_s15.sh && python3 scripts/pmc_mix.py gpurun_out/s33
