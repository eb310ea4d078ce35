#!/bin/bash
# Step tables of the three ResNet-50 trunks at HEAD: tools/prof_headline.sh's passes
# (kernel trace, FETCH_SIZE, WRITE_SIZE, MFMA busy + clock) per trunk; tools/step_table.py turns each
# directory into profiles/<tag>/step_<trunk>.md.  usage: PROF_TAG=x bash tools/prof_trunks.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${PROF_TAG:-trunks}
for cfg in "sw:--trunk sw --precision bf16" "isw:--trunk isw" "ibn:--trunk ibn"; do
  name=${cfg%%:*}; args=${cfg#*:}
  BENCH_EXTRA="$args" PROF_TAG=$T/$name bash tools/prof_headline.sh || exit $?
  echo "$name done"
done
