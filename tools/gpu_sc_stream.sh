#!/bin/bash
# Step time with the smartcrop stage on its own (priority) stream vs the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/scstream
mkdir -p $OUT
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
}
run base FI_SC_STREAM=0
run stream FI_SC_STREAM=1
run prio FI_SC_STREAM=1 FI_SC_PRIO=1
