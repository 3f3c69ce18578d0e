# A/B of two builds of libxerus_amd.so on one box: abtmp/old.so (XRS_LIB_PATH) against the in-tree build,
# alternating. Usage: bash tools/ab_lib.sh OUTDIR [env for tools/trunc_profile.py, e.g. "RANK=128 TARGET=64"]
set -e
O=$1; shift; mkdir -p $O
for k in 1 2 3; do
  env $@ XRS_LIB_PATH=$PWD/abtmp/old.so REPS=8 timeout -k 10 120 python tools/trunc_profile.py > $O/old_$k.txt 2>&1
  env $@ REPS=8 timeout -k 10 120 python tools/trunc_profile.py > $O/new_$k.txt 2>&1
done
tail -n 3 $O/old_*.txt $O/new_*.txt
