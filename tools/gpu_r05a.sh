set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py "tests/test_gpu_parity.py::test_group_policy_same_results" tests/test_gpu_parity.py::test_launch_shape_names_the_kernel tests/test_gpu_parity.py::test_instance_bits_do_not_depend_on_the_batch tests/test_gpu_parity.py::test_iteration_counts_match_cpp_oracle tests/test_gpu_parity.py::test_bench_two_ranks_rehearsal > gpurun_out/r05a/tests.log 2>&1 || { tail -50 gpurun_out/r05a/tests.log; exit 1; }
tail -15 gpurun_out/r05a/tests.log
tools/ab_tree.sh "" 2 && tools/ab_tree.sh "--batch 2048" 2
