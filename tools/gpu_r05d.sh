set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r05d/tests.log 2>&1
grep -E "FAILED|passed|failed" gpurun_out/r05d/tests.log | tail -12
tools/ab_tree.sh "--config 5" 2 ab_base0 . && tools/ab_tree.sh "" 1 ab_base0 .
MPCX_STAMPS_LIB=mpc-verde_amd/mpcx/libmpcx_sub5.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/stamp_profile.py --model pend --N 100 --batch 2048 --steps 3 > gpurun_out/r05d/stamps_c5_sub.json 2> gpurun_out/r05d/stamps_c5_sub.err
MPCX_STAMPS_LIB=mpc-verde_amd/mpcx/libmpcx_sub2.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/stamp_profile.py --steps 3 > gpurun_out/r05d/stamps_c2_sub.json 2> gpurun_out/r05d/stamps_c2_sub.err
python3 -c "import json;d=json.load(open('gpurun_out/r05d/stamps_c5_sub.json'));print(d['cycles_per_iter'], d['share_all_waves'])"
