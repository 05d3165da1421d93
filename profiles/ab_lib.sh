set -e
mkdir -p gpurun_out/ab
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-smooth --steps 3 > gpurun_out/ab/$name.log 2>&1; }
