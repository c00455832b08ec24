# A/B library: babble_amd/libhgx_<tag>.so = the current objects with <file> taken from git <rev>
# usage: bash tools/build_ab.sh TAG REV FILE [FILE...]   (after the main build)
set -e
TAG=$1; REV=$2; shift 2
D=babble_amd/build_ab_$TAG; mkdir -p $D/src
OBJS=""
for o in babble_amd/build/*.o; do
  b=$(basename $o .o)
  skip=0
  for f in "$@"; do [ "$b" = "$f" ] && skip=1; done
  [ $skip = 0 ] && OBJS="$OBJS $o"
done
for f in "$@"; do
  git show $REV:babble_amd/csrc/$f > $D/src/$f
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -Ibabble_amd/csrc -c $D/src/$f -o $D/$f.o
  OBJS="$OBJS $D/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o babble_amd/libhgx_$TAG.so $OBJS
echo built babble_amd/libhgx_$TAG.so
