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
