# One GPU call: the GPU test suite, then a list of bench commands, each under its
# own time limit; stops at the first crash / fault / time-out (exit status other
# than 0 or a test failure), never retries.
# usage: bash tools/gpu_run.sh <tag> [--no-tests] ["ENV=.. python bench.py ..." ...]
set -u
export TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
if [ "${1:-}" = "--no-tests" ]; then shift; else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1
  rc=$?
  tail -3 $O/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
fi
i=0
for cmd in "$@"; do
  i=$((i + 1))
  echo "[$i] $cmd"
  timeout -k 10 600 bash -c "$cmd" > $O/b$i.json 2> $O/b$i.err
  rc=$?
  tail -c 600 $O/b$i.json
  if [ $rc -eq 1 ]; then echo "[$i] rc=1 (failure, not a crash)"; tail -5 $O/b$i.err; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$i] rc=$rc: stop"; tail -5 $O/b$i.err; exit $rc; fi
done
echo done
