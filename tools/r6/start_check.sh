set -o pipefail
mkdir -p gpurun_out/r6s
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6s/pytest_gpu.txt 2>&1 && tail -n 2 gpurun_out/r6s/pytest_gpu.txt &&
timeout -k 10 300 python3 bench.py --steps 600 --warmup 200 > gpurun_out/r6s/bench.json 2> gpurun_out/r6s/bench.err && cut -c1-400 gpurun_out/r6s/bench.json &&
timeout -k 10 200 python3 tools/band_emulate.py --balanced --bands 8 --inflight 3 > gpurun_out/r6s/bands_c4.jsonl 2> gpurun_out/r6s/bands.err && tail -n 1 gpurun_out/r6s/bands_c4.jsonl | cut -c1-600
