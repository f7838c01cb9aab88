#!/bin/bash
# r06f: in-context diagnosis (r06d.sh: clock sampler under the kernel trace, TCC pass) and the C2 bench kernel trace
# of the current tree (sigmoid-logit GELU)
cd "$(dirname "$0")/.."
bash scripts/r06d.sh r06f || exit $?
bash scripts/run.sh r06f trace
