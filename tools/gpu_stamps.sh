#!/bin/bash
# stamps (per-phase cycle shares) of config 2 and config 5 on the diagnostic build, and the
# config-5 bench line: tools/gpu_stamps.sh TAG
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-r04}
timeout -k 10 300 python3 tools/stamp_profile.py --steps 3 > gpurun_out/${T}_stamps_c2.json 2> gpurun_out/${T}_stamps_c2.err || exit 1
timeout -k 10 300 python3 tools/stamp_profile.py --model pend --N 100 --batch 2048 --steps 3 > gpurun_out/${T}_stamps_c5.json 2> gpurun_out/${T}_stamps_c5.err || exit 1
timeout -k 10 300 python3 bench.py --config 5 --no-cpu --no-roofline --no-reference-warm-start > gpurun_out/${T}_b5.json 2> gpurun_out/${T}_b5.err || exit 1
cat gpurun_out/${T}_stamps_c5.json; python3 -c "import json;d=json.loads(open('gpurun_out/${T}_b5.json').read().strip().splitlines()[-1]);print(d['value'],d['lockstep'],d['solve_kernel']['us_per_ipm_iteration'])"
