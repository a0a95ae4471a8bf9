#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box.  Each step has its own time limit; a step
# that faults (abort 134, segfault 139, timeout 124/137, or any signal) ends the session, a
# step whose tests merely fail (exit 1) does not.  Output goes to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== [$name] $(date +%T) $*" | tee -a $OUT/session.log
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== [$name] exit $rc" | tee -a $OUT/session.log
    tail -n 5 "$OUT/$name.log" | tee -a $OUT/session.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "=== stopping: step $name exited $rc" | tee -a $OUT/session.log
        exit $rc
    fi
    return 0
}
i=0
for s in "$@"; do
    i=$((i+1))
    case "$s" in
        smoke)   step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
        pytest)  step pytest 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ;;
        bench)   step bench 600 python bench.py --steps 10 --warmup 3 ;;
        bench10m) step bench10m 600 python bench.py --n 10000000 --steps 5 --warmup 2 --no-adc --no-cpu-baseline --no-alt-data --no-config5 --no-configs ;;
        prof)    step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs --no-config5 --no-north-star ;;
        *)       step "custom$i" 600 bash -c "$s" ;;
    esac
done
echo "=== session done $(date +%T)" | tee -a $OUT/session.log
