#!/bin/bash
# gpurun with a pre-push check: the in-tree libdanse_mi355x.so must be newer
# than every source it is built from (danse_amd.build.up_to_date), otherwise
# the box would run a stale library (round 4's r4e lease).
#   scripts/gpurun.sh TIMEOUT_S 'command ...'
set -e
cd "$(dirname "$0")/.."
python -c "import sys; from danse_amd import build; sys.exit(0 if build.up_to_date() else 1)" \
  || { echo "libdanse_mi355x.so is stale: run python -c 'from danse_amd import build; build.build()'"; exit 3; }
T=$1
shift
exec /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
