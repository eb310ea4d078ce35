#!/bin/bash
# Run GPU steps in order, each "TIMEOUT_S OUTFILE CMD..." as one argument string; stop at the
# first step that timed out, aborted or crashed (rc 124/134/137/139 or > 128); an ordinary
# failure (e.g. pytest rc 1) is reported and the next step runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for step in "$@"; do
  t=${step%% *}; rest=${step#* }; out=${rest%% *}; cmd=${rest#* }
  mkdir -p "$(dirname "$out")"
  echo "== $cmd  (limit ${t}s, -> $out)"
  timeout -k 10 "$t" bash -c "$cmd" > "$out" 2>&1
  rc=$?
  echo "   rc $rc; tail:"; tail -4 "$out" | sed 's/^/   /'
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "stopping: step ended abnormally"; exit $rc
  fi
done
