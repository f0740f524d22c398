# Build an A/B variant of the library:
#   bash tools/build_variant.sh NAME "-DFLAG ..."            -> build/libmrgpu_NAME.so (working tree)
#   REV=<git rev> bash tools/build_variant.sh NAME [flags]   -> the sources of that commit
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
flags="$*"
tmp=$HERE/build/var_$name
rm -rf $tmp && mkdir -p $tmp
src=$HERE/csrc
inc=$HERE/../include
if [ -n "$REV" ]; then  # the sources of a past commit (headers included)
  git -C $HERE/.. archive "$REV" distributed-systems-implemented_amd/csrc include | tar -x -C $tmp
  src=$tmp/distributed-systems-implemented_amd/csrc
  inc=$tmp/include
fi
for f in $(ls $src/*.hip | xargs -n1 basename | sed 's/\.hip$//'); do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -w -I$inc $flags -c $src/$f.hip -o $tmp/$f.o &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -o $HERE/build/libmrgpu_$name.so $tmp/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-soname,libmrgpu.so
rm -rf $tmp
echo built $HERE/build/libmrgpu_$name.so
