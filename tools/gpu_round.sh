#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprofv3 kernel-trace summary of the bench command,
# and the HBM-traffic PMC passes of the roofline kernel.  Every GPU step has its own time limit and
# the first failure ends the script.
#   gpurun --timeout 1100 -- 'bash tools/gpu_round.sh <tag> [steps...]'   (steps: test smoke bench prof pmc)
TAG=${1:-run}
shift
STEPS=${*:-"test bench prof pmc"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1

step() { case " $STEPS " in *" $1 "*) return 0 ;; esac; return 1; }

if step test; then
    echo "== pytest -m gpu"
    (cd "$R" && timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$O/pytest_gpu.log" 2>&1)
    rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
if step smoke; then
    echo "== smoke"
    (cd "$R" && timeout -k 10 300 python -u __graft_entry__.py smoke > "$O/smoke.log" 2>&1)
    rc=$?; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if step bench; then
    echo "== bench"
    (cd "$R" && timeout -k 10 400 python -u bench.py > "$O/bench.log" 2>&1)
    rc=$?; tail -1 "$O/bench.log"; [ $rc -eq 0 ] || exit $rc
fi
if step parts; then
    echo "== part timing"
    (cd "$R" && timeout -k 10 300 python -u tools/part_timing.py > "$O/parts.log" 2>&1)
    rc=$?; cat "$O/parts.log" | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
fi
if step prof; then
    echo "== rocprofv3 kernel trace of the bench command"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
        -- python3 "$R/bench.py" --no-cpu-baseline > "$O/prof_bench.log" 2>&1
    rc=$?; tail -1 "$O/prof_bench.log"; [ $rc -eq 0 ] || exit $rc
    f=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
    python3 "$R/profiles/prof_summary.py" "$(dirname "$f")" 45 > "$O/prof_summary.txt" 2>&1
    head -50 "$O/prof_summary.txt"
    ms=$(python3 -c "import json,sys; print(json.loads([l for l in open('$O/prof_bench.log') if l.startswith('{')][-1])['ms_per_step'])")
    t=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
    python3 "$R/profiles/step_breakdown.py" "$t" "$ms" > "$O/step_breakdown.txt" 2>&1; cat "$O/step_breakdown.txt"
    rm -f "$t"     # (the full trace exceeds what gpurun_out carries back)
fi
if step c4; then
    echo "== C4 bench (512^2 3-ch, cbase 32768, bs16, fp16)"
    (cd "$R" && timeout -k 10 500 python -u bench.py --res 512 --batch-gpu 16 --img-channels 3 --cbase 32768 --c-dim 0 \
        > "$O/c4_bench.log" 2>&1)
    rc=$?; tail -1 "$O/c4_bench.log"; [ $rc -eq 0 ] || exit $rc
fi
if step c5; then
    echo "== C5 bench (1024^2 3-ch, cbase 32768, bs8, bf16)"
    (cd "$R" && timeout -k 10 500 python -u bench.py --res 1024 --batch-gpu 8 --img-channels 3 --cbase 32768 --c-dim 0 \
        --fp16-dtype bf16 > "$O/c5_bench.log" 2>&1)
    rc=$?; tail -1 "$O/c5_bench.log"; [ $rc -eq 0 ] || exit $rc
fi
if step pmc; then
    # HBM bytes of the roofline kernel: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots).
    for c in FETCH_SIZE WRITE_SIZE; do
        echo "== pmc $c"
        timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'conv3x3_(halo|c64p|c64r)' -d "$O/pmc_$c" -o run \
            --output-format csv -- python3 "$R/tools/roofline_only.py" > "$O/pmc_$c.log" 2>&1
        rc=$?; tail -1 "$O/pmc_$c.log"; [ $rc -eq 0 ] || exit $rc
    done
    python3 "$R/tools/pmc_traffic.py" "$O" "$O/roofline_traffic.json" > "$O/pmc_traffic.txt" 2>&1; cat "$O/pmc_traffic.txt"
fi
if step diag; then
    # where the halo conv waves wait (one pass, 8 SQ counters; MI355X_MICROARCH.md rocprofv3 PMC slots)
    echo "== pmc diag halo"
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex 'conv3x3|conv_fwd|wgrad' \
        -d "$O/diag" -o run --output-format csv -- python3 "$R/tools/conv_micro.py" --reps 3 > "$O/diag.log" 2>&1
    rc=$?; tail -5 "$O/diag.log"; [ $rc -eq 0 ] || exit $rc
fi
if step mem; then
    echo "== memory-path microbenchmarks"
    (cd "$R" && timeout -k 10 120 python -u tools/membench.py > "$O/mem.log" 2>&1)
    rc=$?; grep -v amdgpu.ids "$O/mem.log"; [ $rc -eq 0 ] || exit $rc
fi
if step trace; then
    echo "== kernel trace of the iteration's parts and loss phases"
    timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/tr" -o run --output-format csv \
        -- python3 "$R/tools/trace_parts.py" > "$O/trace.log" 2>&1
    rc=$?; tail -1 "$O/trace.log"; [ $rc -eq 0 ] || exit $rc
    python3 "$R/tools/trace_report.py" "$O/tr" 30 > "$O/trace_report.txt" 2>&1; grep "===" "$O/trace_report.txt"
fi
if step micro; then
    echo "== conv micro"
    (cd "$R" && timeout -k 10 300 python -u tools/conv_micro.py > "$O/micro.log" 2>&1)
    rc=$?; grep -v amdgpu.ids "$O/micro.log"; [ $rc -eq 0 ] || exit $rc
fi
if step calib; then
    # FETCH_SIZE calibration for the C=64 conv's half-line reads (tools/pmc_calib.py)
    for lib in default d3; do
        for c in FETCH_SIZE WRITE_SIZE; do
            echo "== calib $lib $c"
            if [ $lib = default ]; then unset SG2HIP_LIB; else export SG2HIP_LIB="$R/tools/diag_libs/libsg2hip_$lib.so"; fi
            timeout -s KILL 120 rocprofv3 --pmc $c -d "$O/calib_${lib}_$c" -o run --output-format csv \
                -- python3 "$R/tools/pmc_calib.py" > "$O/calib_${lib}_$c.log" 2>&1
            rc=$?; tail -1 "$O/calib_${lib}_$c.log"; [ $rc -eq 0 ] || exit $rc
        done
    done
    unset SG2HIP_LIB
fi
if step var; then
    echo "== c64p variants: $VARS"
    (cd "$R" && bash tools/c64p_var.sh run > "$O/var.log" 2>&1)
    rc=$?; cat "$O/var.log"; [ $rc -eq 0 ] || exit $rc
fi
if step wgswz; then
    echo "== wgrad LDS swizzle A/B"
    (cd "$R" && for sw in 0 1 0 1; do echo "SWZ=$sw"; SG2_WGRAD_SWZ=$sw timeout -k 10 120 python3 -u tools/wgrad_s2_ab.py || exit 1; done > "$O/wgswz.log" 2>&1)
    rc=$?; grep -v amdgpu.ids "$O/wgswz.log"; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"
