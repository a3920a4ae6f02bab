#!/bin/bash
# Run GPU steps in order, each under its own time limit: "name|seconds|command" per argument.  A step that
# fails with exit status 1 (test failures) is recorded and the next step runs; any other non-zero status
# (fault, abort, signal, time limit) ends the script there.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/steps
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    echo "== $name ($secs s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
    rc=$?
    grep -v "amdgpu.ids" "$O/$name.log" | tail -15
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo "== done"
