# Build an A/B variant of the library with extra compile flags:
#   bash tools/build_variant.sh NAME "-DFLAG ..."   -> build/libmrgpu_NAME.so
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
flags="$*"
tmp=$HERE/build/var_$name
mkdir -p $tmp
for f in mrgpu_map mrgpu_wc mrgpu_reduce mrgpu_json mrgpu_api; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -w $flags -c $HERE/csrc/$f.hip -o $tmp/$f.o &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -o $HERE/build/libmrgpu_$name.so $tmp/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-soname,libmrgpu.so
rm -rf $tmp
echo built $HERE/build/libmrgpu_$name.so
