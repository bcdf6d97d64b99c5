# A/B timings of the scoring pipeline's switches (FraudPipeline env switches), bench lines to
# gpurun_out/<tag>_ab_<name>.json.  usage: bash tools/gpu_ab.sh <tag>
set -eu
TAG=${1:?tag}
mkdir -p gpurun_out
run() {  # run <name> <env assignments...>
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 \
        > gpurun_out/${TAG}_ab_${name}.json 2>> gpurun_out/${TAG}_ab.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_ab_${name}.json')); print('${name}', d['ms_per_step'], [(r['stage'], r['ms_in_step']) for r in d['kernels']['per_stage']])"
}
for spec in ${AB_RUNS:-base:FDX_OVERLAP=1}; do
    name=${spec%%:*}
    IFS=, read -ra kv <<< "${spec#*:}"
    run "$name" "${kv[@]}"
done
echo ab done
