#!/bin/bash
# A/B libraries: tools/ab_build.sh NAME [extra hipcc flags...] — libdq.so with freq.hip / strings.hip / scan.hip / kll.hip compiled with the
# given -D flags (or from a git revision: FREQ_REV / STR_REV / SCAN_REV / KLL_REV; CAST_SRC=path for cast.hip), into tools/ab/NAME.so (select with DQ_LIBRARY).
set -eu
cd "$(dirname "$0")/../deequ_amd/csrc"
NAME=$1; shift
OUT=../../tools/ab
mkdir -p $OUT/$NAME.build
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function"
objs=""
for f in dq_api.cpp host_algebra.cpp multi.cpp scan.hip predicate.hip synth.hip freq.hip quantile.hip strings.hip regex.hip kll.hip cast.hip; do
  src=$f
  if [ "$f" = freq.hip ] && [ -n "${FREQ_REV:-}" ]; then git show "$FREQ_REV:deequ_amd/csrc/freq.hip" > _ab_rev_freq.hip; src=_ab_rev_freq.hip; fi
  if [ "$f" = strings.hip ] && [ -n "${STR_REV:-}" ]; then git show "$STR_REV:deequ_amd/csrc/strings.hip" > _ab_rev_strings.hip; src=_ab_rev_strings.hip; fi
  if [ "$f" = scan.hip ] && [ -n "${SCAN_REV:-}" ]; then git show "$SCAN_REV:deequ_amd/csrc/scan.hip" > _ab_rev_scan.hip; src=_ab_rev_scan.hip; fi
  if [ "$f" = kll.hip ] && [ -n "${KLL_REV:-}" ]; then git show "$KLL_REV:deequ_amd/csrc/kll.hip" > _ab_rev_kll.hip; src=_ab_rev_kll.hip; fi
  if [ "$f" = cast.hip ] && [ -n "${CAST_SRC:-}" ]; then cp "$CAST_SRC" _ab_src_cast.hip; src=_ab_src_cast.hip; fi
  case $f in freq.hip|strings.hip|scan.hip|kll.hip|cast.hip|quantile.hip) /opt/rocm/bin/hipcc $FLAGS "$@" -I. -x hip -c $src -o $OUT/$NAME.build/$f.o ;; *) cp build/$f.o $OUT/$NAME.build/$f.o ;; esac
  objs="$objs $OUT/$NAME.build/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/$NAME.so $objs -ldl
rm -rf $OUT/$NAME.build _ab_rev_freq.hip _ab_rev_strings.hip _ab_rev_scan.hip _ab_rev_kll.hip _ab_src_cast.hip
echo built $OUT/$NAME.so
