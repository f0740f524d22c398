# One GPU-box command for every measurement run (replaces the per-run
# gpu_rNN*.sh scripts of rounds 1-5).  Steps run in order, each under its own
# time limit, and the first failure ends the run (set -e: nothing more touches
# the GPU after a fault, an abort or a time limit).
#
#   bash distributed-systems-implemented_amd/tools/gpu_run.sh OUT STEP [STEP ...]
#
# STEP:
#   tests[=K]          pytest -m gpu (optionally -k K) -> OUT/tests.log
#   smoke              __graft_entry__.smoke()         -> OUT/smoke.log
#   bench=NAME[:ARGS]  python bench.py ARGS            -> OUT/NAME.json / .err
#                      (ARGS: flags joined by colons, e.g.
#                       bench=c5:--workload:c5:--no-cpu-baseline)
#   prof=W[:ARGS]      rocprofv3 kernel-trace summary of bench.py --workload W
#   pmc=NAME[:ARGS]    SQ / FETCH_SIZE / WRITE_SIZE passes over mapprobe.py ARGS
#                      (pmc_passes.sh)                 -> OUT/pmc_NAME/
#   probe=ARGS         tools/mapprobe.py ARGS          -> OUT/mapprobe.jsonl
#   ab=W:A:B[:...]     alternating A/B of build/libmrgpu_<A|B>.so (ab_libs.sh)
set -e
out=gpurun_out/${1:?usage: gpu_run.sh OUT STEP...}
shift
mkdir -p "$out"
tools=distributed-systems-implemented_amd/tools
rest() { local r=${1#*:}; [ "$r" = "$1" ] && r=""; printf '%s' "$r"; }  # ARGS after NAME:
for step in "$@"; do
    verb=${step%%=*}
    arg=${step#*=}
    [ "$arg" = "$step" ] && arg=""
    echo "[gpu_run] $(date +%T) $step"
    case $verb in
    tests)
        k=()
        [ -n "$arg" ] && k=(-k "$arg")
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${k[@]}" \
            > "$out/tests.log" 2>&1
        tail -2 "$out/tests.log"
        ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
        tail -1 "$out/smoke.log"
        ;;
    bench)
        name=${arg%%:*}
        IFS=: read -r -a bargs <<< "$(rest "$arg")"
        timeout -k 10 600 python -u bench.py "${bargs[@]}" > "$out/$name.json" 2> "$out/$name.err"
        python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d.get('value'),d.get('ms_per_step'),d.get('roofline',{}).get('frac'),d.get('phases_ms'),d.get('checks',{}).get('exact_vs_oracle'))" "$out/$name.json" "$name"
        ;;
    prof)
        w=${arg%%:*}
        IFS=: read -r -a bargs <<< "$(rest "$arg")"
        timeout -k 10 450 bash $tools/prof_bench.sh "${out#gpurun_out/}/prof_$w" "$w" "${bargs[@]}"
        ;;
    pmc)
        name=${arg%%:*}
        IFS=: read -r -a pargs <<< "$(rest "$arg")"
        timeout -k 10 600 bash $tools/pmc_passes.sh "$out/pmc_$name" "${pargs[@]}"
        ;;
    probe)
        IFS=: read -r -a pargs <<< "$arg"
        timeout -k 10 400 python -u $tools/mapprobe.py "${pargs[@]}" >> "$out/mapprobe.jsonl" 2>> "$out/mapprobe.err"
        tail -3 "$out/mapprobe.jsonl"
        ;;
    ab)
        IFS=: read -r -a abargs <<< "$arg"
        timeout -k 10 900 bash $tools/ab_libs.sh "${out#gpurun_out/}" "${abargs[@]}"
        ;;
    *)
        echo "gpu_run: unknown step $step" >&2
        exit 2
        ;;
    esac
done
