# Round-end measurement set: the bench lines of configs 2-5, the headline under rocprofv3 --stats, smoke().
set -o pipefail
bash tools/gpu_step.sh bench:head,--steps,20,--warmup,5 bench:models,--workload,models,--no-cpu \
    bench:sample,--workload,sample,--no-cpu bench:fit,--workload,fit,--no-cpu,--fit-max-seconds,30 \
    stats:head,--steps,50,--warmup,5,--no-cpu || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
