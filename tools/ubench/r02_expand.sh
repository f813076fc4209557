#!/bin/bash
# Expand conv (config-4 shape, B = 65,536 windows): the library's RB choice and RB 1/2/4,
# each with stores on (0) and off (2).
set -o pipefail
cd "$(dirname "$0")"
for rb in ${RBS:-0 1 2 4}; do
  timeout -k 5 120 ./expand_check ${B:-65536} $rb ${ABL:-0 2} || exit $?
done
