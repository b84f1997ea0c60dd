set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench_train.py --steps 8 --warmup 2 > gpurun_out/gc_on_$i.log 2>&1 && \
timeout -k 10 300 python -c "import gc,sys,runpy; gc.disable(); sys.argv=['bench_train.py','--steps','8','--warmup','2']; runpy.run_path('bench_train.py', run_name='__main__')" > gpurun_out/gc_off_$i.log 2>&1 || exit 1
done
