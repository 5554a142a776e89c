set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04av
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04av/gpu_tests.txt 2>&1 && tail -3 gpurun_out/r04av/gpu_tests.txt &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04av/smoke.txt 2>&1 && tail -1 gpurun_out/r04av/smoke.txt &&
timeout -k 10 300 python bench.py > gpurun_out/r04av/bench.json 2> gpurun_out/r04av/bench.err && cut -c1-400 gpurun_out/r04av/bench.json
