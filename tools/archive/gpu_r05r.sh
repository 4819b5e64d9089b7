#!/bin/bash
# round 5, pass r: full GPU suite + smoke + bench at HEAD
set -u
bash tools/gpu_suite.sh r05r || exit 1
