#!/bin/bash
# round 6: final profiles (kernel trace + PMC passes) for the given configs
set -o pipefail
for cfg in "$@"; do
  timeout -k 10 560 tools/profile.sh r06_$cfg --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-extra || { echo "profile $cfg failed"; exit 1; }
done
echo done
