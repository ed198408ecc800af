export TMPDIR=/tmp
tools/gpu_step.sh jtests 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "join" && \
tools/gpu_step.sh jbench 300 python -u bench.py --workload join --steps 10 --warmup 3 && \
tools/gpu_step.sh jstats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/jprof -o join --output-format csv -- python -u bench.py --workload join --steps 5 --warmup 1 --no-verify --no-cpu-baseline
