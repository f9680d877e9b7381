for i in 1 2; do
for n in 25 1; do
MPCX_UNICYCLE_SCAN_MIN_N=$n timeout -k 10 200 python3 bench.py --config 2 --no-cpu --no-roofline 2>/dev/null | python3 -c "import json,sys;d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]);print('minN=$n', d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'])"
done; done
