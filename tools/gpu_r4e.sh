timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4e_tests.log 2>&1; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/zopt_iter_probe.py 4 > gpurun_out/r4e_probe.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4e_smoke.log 2>&1 || exit $?
ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so AB_VARIANTS=64,65,66,50 AB_HW=148 AB_ROUNDS=4 timeout -k 10 200 python -u tools/x3_ab.py > gpurun_out/r4e_x3ab.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_DCONV_PRESPLIT 0 1 || exit $?
timeout -k 10 400 python -u tools/grid_c3_ab.py base gstep_x6 gstep_f32 head_x6 bias64 gstep_x6+head_x6+bias64 > gpurun_out/r4e_grid.log 2>&1
