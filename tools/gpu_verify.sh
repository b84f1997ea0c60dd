# One parameterised GPU lease (replaces the per-call gpu_r4*.sh scripts): bash tools/gpu_verify.sh TAG [STEPS...]
# STEPS (default: tests smoke bench): tests = every -m gpu test, smoke = __graft_entry__.smoke(), bench = the default
# bench line, c2prof = tools/prof_bench.sh --no-legs + its summary (profiles-ready files under gpurun_out/TAG_c2*).
# Each step under its own time limit, outputs in gpurun_out/TAG_<step>.log; the first failing step ends the lease.
set -o pipefail
tag=$1; shift
steps=${*:-tests smoke bench}
mkdir -p gpurun_out
for s in $steps; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread \
             > gpurun_out/${tag}_tests.log 2>&1 || exit $? ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
             > gpurun_out/${tag}_smoke.log 2>&1 || exit $? ;;
    bench) timeout -k 10 400 python3 bench.py > gpurun_out/${tag}_bench.log 2>&1 || exit $? ;;
    c2prof) bash tools/prof_bench.sh gpurun_out/${tag}_prof --no-legs || exit $?
            python3 tools/prof_summary.py gpurun_out/${tag}_prof gpurun_out/${tag}_c2 > gpurun_out/${tag}_summary.log 2>&1 || exit $?
            rm -rf gpurun_out/${tag}_prof/pmc_fetch gpurun_out/${tag}_prof/pmc_write ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
