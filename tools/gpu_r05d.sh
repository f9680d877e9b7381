set -o pipefail
L=mpc-verde_amd/mpcx
for i in 1 2; do for lib in libmpcx libmpcx_redo1 libmpcx_galld; do
  MPCX_LIB=$L/$lib.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 bench.py --config 5 --no-cpu --no-roofline --no-reference-warm-start > gpurun_out/ab5_${lib}_$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab5_${lib}_$i.json') if l.startswith('{')][-1]);print('$lib', d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'], d['solve_kernel']['timed_launch_ms'])"
done; done
(cd ab_base0 && timeout -k 10 200 python3 bench.py --config 5 --no-cpu --no-roofline --no-reference-warm-start > ../gpurun_out/ab5_base0.json 2>/dev/null; python3 -c "import json;d=json.loads([l for l in open('../gpurun_out/ab5_base0.json') if l.startswith('{')][-1]);print('base0', d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'], d['solve_kernel']['timed_launch_ms'])")
