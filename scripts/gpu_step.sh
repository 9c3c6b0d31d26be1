set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.txt 2>&1 && tail -2 gpurun_out/gpu_tests.txt && \
TAG=r06d PROFILE=1 PROF_LEGS="headline" timeout -k 10 900 bash scripts/gpu_bench.sh > gpurun_out/prof_final.log 2>&1 && tail -2 gpurun_out/prof_final.log && \
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r06d.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels'], d['zstd']['value'], d['deflate']['value'], d['deflate_dynamic']['value'])"
