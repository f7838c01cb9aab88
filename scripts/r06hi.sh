#!/bin/bash
# r06h (fp16 / bf16 C2 parity, fp8 tests, C4 LayerNorm rows-per-wave A/B) then r06i (halo transform-tap A/B)
cd "$(dirname "$0")/.."
bash scripts/r06h.sh || exit $?
bash scripts/r06i.sh
