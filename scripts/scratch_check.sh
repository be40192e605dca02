#!/bin/bash
# scratch bytes / VGPRs per k_decode_pipe kernel of a decode.hip (default: the working copy)
SRC=${1:-oxidized-mtbl_amd/csrc/decode.hip}
shift
OUT=$(mktemp /tmp/dec.XXXX.s)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ioxidized-mtbl_amd/csrc "$@" --cuda-device-only -S "$SRC" -o "$OUT" || exit 1
awk '/\.amdhsa_kernel /{k=$2} /amdhsa_private_segment_fixed_size/{s=$2} /amdhsa_next_free_vgpr/{print substr(k,1,70), "scratch", s, "vgpr", $2}' "$OUT"
rm -f "$OUT"
