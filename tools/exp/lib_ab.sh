#!/bin/bash
# library-build A/B for the front: rmb_front3 phase cycles per build (front_prof.py), then
# interleaved pipeline rounds (ab3.sh).  usage: lib_ab.sh TAG ROUNDS SUFFIX...  (SUFFIX "" =
# libtrk_amd.so, else libtrk_amd_SUFFIX.so next to it)
set -o pipefail
TAG=$1; N=$2; shift 2
LIB=${GRAFT_REPO_ROOT:-$(pwd)}/a-lightweight-unsupervised-feature-extractor-_amd
mkdir -p gpurun_out
ENVS=()
for sfx in "$@"; do
  E=""; [ -n "$sfx" ] && E="TRK_LIB_PATH=$LIB/libtrk_amd_$sfx.so"
  ENVS+=("$E")
  env $E timeout -k 10 120 python tools/exp/front_prof.py "" > "gpurun_out/${TAG}_prof_${sfx:-base}.txt" 2>&1 || { echo "prof $sfx failed"; exit 1; }
  echo "== ${sfx:-base}"; grep '"variant"' "gpurun_out/${TAG}_prof_${sfx:-base}.txt" | cut -c1-330
done
bash tools/exp/ab3.sh "$TAG" "$N" "${ENVS[@]}"
