#!/bin/bash
# Samples the GPU's power and clocks (rocm-smi) while a workload runs on it, to tell whether a
# phase is power/clock-limited.  Usage: tools/power_probe.sh OUTDIR -- cmd...
OUT=$1; shift; shift
mkdir -p "$OUT"
"$@" > "$OUT/workload.log" 2>&1 &
pid=$!
sleep 3
for i in $(seq 1 40); do
  kill -0 $pid 2>/dev/null || break
  { date +%s.%N; timeout -k 2 5 rocm-smi --showpower --showclocks --showtemp --showuse 2>&1; } >> "$OUT/smi.log"
  sleep 0.2
done
wait $pid
echo "workload rc=$?"
