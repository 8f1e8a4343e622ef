#!/bin/bash
# Throwaway library variants for on-box A/B timing (round 5): each is the
# in-tree csrc with one change, built into _ab/<name>/libmicall_hip.so
# (git-ignored; shipped to the GPU box with the tree).  Run with
#   bash profiles/diag/ab_bench.sh ROUNDS name ...   (MICALL_HIP_LIB per variant)
set -e
cd "$(dirname "$0")/../.."
build() {   # name, python patch (applied to the copied sources)
  local name=$1 patch=$2 src=micall-lite_amd/_abv_$1
  rm -rf "$src"; cp -r micall-lite_amd/csrc "$src"; rm -rf "$src/_obj"
  (cd "$src" && python3 -c "$patch")
  mkdir -p "_ab/$name"
  make -s -j8 -C "$src" OUT="$PWD/_ab/$name/libmicall_hip.so" OBJDIR=_obj > /dev/null
  rm -rf "$src"
  echo "built _ab/$name"
}
# k_dp without the next-group prefetch of the score words in dp_pair
build noprefetch '
s = open("mh_map.hip").read()
a = s.index("    // the next group'"'"'s score words and reference codes are read while this")
b = s.index("        uint32_t acc = 0;", a)
s = s[:a] + """    for (int i0 = 0; i0 < mhi; i0 += 8) {
        uint32_t tbv[8];
        int rcv[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            tbv[t] = tab[i0 + t];
            rcv[t] = refw[i0 + t];
        }
""" + s[b:]
open("mh_map.hip", "w").write(s)
'
# reads of 257-320 rows staged in rounds (no LDS-DMA prefetch), waves per
# workgroup still chosen for residency
build multiround '
s = open("mh_map.hip").read()
s = s.replace("rows_pad <= 256 ? RawLayout<256>::BYTES : rows_pad <= 320 ? RawLayout<320>::BYTES : 0",
              "rows_pad <= 256 ? RawLayout<256>::BYTES : 0")
s = s.replace("const int round = rows_pad <= 256 ? 256 : rows_pad <= 320 ? 320 : 0;",
              "const int round = rows_pad <= 256 ? 256 : 0;")
open("mh_map.hip", "w").write(s)
'
