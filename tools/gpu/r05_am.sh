#!/bin/bash
# round 5, call AM: full verification of the build after lg_linear_cat_ffn (GPU suite, smoke, bench, round profile)
set -o pipefail
OUT=r05v6 bash tools/gpu/r05_verify.sh
