#!/bin/bash
# round 5, pass af: full GPU suite + smoke + bench at HEAD
set -u
bash tools/gpu_suite.sh r05af || exit 1
