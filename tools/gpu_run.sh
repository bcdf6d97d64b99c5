# One parametrised GPU round trip (through gpurun).  Every GPU step runs under its own time
# limit; the first failure ends the script (nothing more touches the GPU after it).
# usage: bash tools/gpu_run.sh <tag> <step> [<step> ...]
#   tests[=<pytest selection>]   pytest -m gpu (default: tests)
#   smoke                        __graft_entry__.smoke()
#   bench[=<bench.py args>]      one bench.py line  -> <tag>_bench.json
#   trace[=<bench.py args>]      rocprofv3 kernel trace + stats of bench.py -> <tag>_trace/
#   pmc=<counters>[@<args>]      one rocprofv3 --pmc pass of bench.py -> <tag>_pmc_<n>/
#   forest[=<bench_forest args>] bench_forest.py (configs[2])
#   stream[=<bench_stream args>] bench_stream.py (configs[4])
#   py=<script args>             python3 <script args> (a study script)
#   tracepy=<script args>        rocprofv3 kernel trace + stats of python3 <script args> -> <tag>_tracepy_<n>/
set -eu
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
n=0
for st in "$@"; do
    n=$((n + 1))
    name=${st%%=*}
    arg=""
    [ "$name" != "$st" ] && arg=${st#*=}
    case $name in
    tests)
        timeout -k 10 1000 python -u -m pytest ${arg:-tests} -m gpu -x -v --timeout 400 --timeout-method thread \
            > $O/pytest_$n.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_$n.log; exit 1; }
        tail -3 $O/pytest_$n.log ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
            || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
        cat $O/smoke.log ;;
    bench)
        timeout -k 10 600 python -u bench.py $arg > $O/bench_$n.json 2> $O/bench_$n.err \
            || { echo "bench failed"; tail -30 $O/bench_$n.err; exit 1; }
        head -c 1500 $O/bench_$n.json; echo ;;
    trace)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n \
            -- python3 bench.py ${arg:---steps 5 --warmup 2 --no-cpu-baseline} > $O/trace_$n.log 2>&1 \
            || { echo "trace failed"; tail -20 $O/trace_$n.log; exit 1; }
        echo "trace $n ok" ;;
    tracepy)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tracepy_$n \
            -- python3 $arg > $O/tracepy_$n.log 2>&1 || { echo "tracepy failed"; tail -20 $O/tracepy_$n.log; exit 1; }
        tail -3 $O/tracepy_$n.log ;;
    pmc)
        ctr=${arg%%@*}
        bargs="--steps 2 --warmup 1 --no-cpu-baseline --isolated-steps 0"
        [ "$ctr" != "$arg" ] && bargs=${arg#*@}
        timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_$n \
            -- python3 bench.py $bargs > $O/pmc_$n.log 2>&1 || { echo "pmc $ctr failed"; tail -20 $O/pmc_$n.log; exit 1; }
        echo "pmc $n ($ctr) ok" ;;
    forest)
        timeout -k 10 600 python -u bench_forest.py $arg > $O/forest_$n.json 2> $O/forest_$n.err \
            || { echo "bench_forest failed"; tail -30 $O/forest_$n.err; exit 1; }
        head -c 1500 $O/forest_$n.json; echo ;;
    stream)
        timeout -k 10 600 python -u bench_stream.py $arg > $O/stream_$n.json 2> $O/stream_$n.err \
            || { echo "bench_stream failed"; tail -30 $O/stream_$n.err; exit 1; }
        head -c 1500 $O/stream_$n.json; echo ;;
    py)
        timeout -k 10 600 python -u $arg > $O/py_$n.log 2>&1 || { echo "py $arg failed"; tail -30 $O/py_$n.log; exit 1; }
        tail -30 $O/py_$n.log ;;
    *)
        echo "unknown step $st"; exit 2 ;;
    esac
done
echo "$TAG done"
