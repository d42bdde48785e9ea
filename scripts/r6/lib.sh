# step NAME SECONDS CMD...: runs one GPU step under its own time limit, output to $O/NAME.log.
# A failing test (exit 1 / 2) is recorded and the script goes on; a time limit, abort or fault
# (124 / 137 / 134 / 139 / other >= 124) ends the script there.
step() {
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(tail -1 "$O/$name.log" | cut -c1-240)"
  if [ $rc -ge 124 ]; then
    echo "[$name] stopping: time limit / abort / fault"
    exit $rc
  fi
  return 0
}

# prof NAME SECONDS OUTDIR_STEPS [bench args]: rocprofv3 kernel trace of bench.py, the per-step timeline
# (scripts/timeline.py) kept, the raw trace deleted (gpurun copies back at most 64 MiB)
prof() {
  local name=$1 secs=$2 steps=$3
  shift 3
  step $name $secs bash scripts/profile_step.sh $O/$name "$@"
  local f
  f=$(ls $O/$name/*/*kernel_trace.csv 2>/dev/null | head -1)
  if [ -n "$f" ]; then
    python3 scripts/timeline.py "$f" $steps > $O/$name.timeline.txt 2>&1
    head -12 $O/$name.timeline.txt
    tail -2 $O/$name.timeline.txt
    rm -f "$f"
  fi
}
