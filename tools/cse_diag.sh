# Diagnostic of the MachineCSE-off experiment: determinism of the product and experiment builds on the
# 6-state bicycle (tools/bits_compare.py dyn, twice each), their per-array differences, and the oracle-
# agreement test on the experiment library (build it with tools/exp_build.sh cse dyn_bicycle -mllvm -disable-machine-cse).
set -o pipefail
L0=$PWD/mpc-verde_amd/mpcx/libmpcx.so; L1=$PWD/mpc-verde_amd/mpcx/libmpcx_cse.so
for i in 1 2; do
  MPCX_LIB=$L0 MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 tools/bits_compare.py dyn /tmp/d0_$i.npz > /dev/null 2>&1 || exit 1
  MPCX_LIB=$L1 MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 tools/bits_compare.py dyn /tmp/d1_$i.npz > /dev/null 2>&1 || exit 1
done
echo "base run1 vs run2: $(python3 tools/bits_compare.py --diff /tmp/d0_1.npz /tmp/d0_2.npz | tr '\n' ' ')"
echo "cse run1 vs run2: $(python3 tools/bits_compare.py --diff /tmp/d1_1.npz /tmp/d1_2.npz | tr '\n' ' ')"
echo "base vs cse: $(python3 tools/bits_compare.py --diff /tmp/d0_1.npz /tmp/d1_1.npz | tr '\n' ' ')"
python3 - <<'PY'
import numpy as np
a,b=np.load('/tmp/d0_1.npz'),np.load('/tmp/d1_1.npz')
for k in a.files:
    x,y=a[k],b[k]
    if x.shape!=y.shape: print(k,'shape',x.shape,y.shape); continue
    if x.dtype.kind=='f':
        d=np.abs(x-y); n=np.sum(~((x==y)|(np.isnan(x)&np.isnan(y))))
        print(k, x.shape, 'n_diff', int(n), 'max_abs', float(np.nanmax(d)) if d.size else 0)
    else:
        print(k, x.shape, 'n_diff', int(np.sum(x!=y)))
PY
MPCX_LIB=$L1 MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider "tests/test_gpu_resto.py::test_config4_dyn_bicycle_batch_vs_ipopt_oracle" 2>&1 | tail -5
