# A/B of library builds on one box: every abtmp/<name>.so (XRS_LIB_PATH; name "old" = the baseline) and the
# in-tree build ("new"), alternating, 3 rounds. Usage: bash tools/ab_lib.sh OUTDIR [env for
# tools/trunc_profile.py, e.g. "RANK=128 TARGET=64"]
set -e
O=$1; shift; mkdir -p $O
for k in 1 2 3; do
  for lib in abtmp/*.so; do
    b=$(basename $lib .so)
    env $@ XRS_LIB_PATH=$PWD/$lib REPS=8 timeout -k 10 120 python tools/trunc_profile.py > $O/${b}_$k.txt 2>&1
  done
  env $@ REPS=8 timeout -k 10 120 python tools/trunc_profile.py > $O/new_$k.txt 2>&1
done
tail -n 3 $O/*_[123].txt
