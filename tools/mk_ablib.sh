#!/bin/bash
# Build an A/B library: the current objects (build/dvie, `make` first) with one source file
# taken from a git revision instead.  usage: bash tools/mk_ablib.sh <csrc file.hip> <rev> <out.so>
set -e
f=$1; rev=$2; out=$3
src=deep_video_interpolation_extrapolation_amd/csrc
tmp=$(mktemp -d)
git show "$rev:$src/$f" > $tmp/$f
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -I $src -c $tmp/$f -o $tmp/${f%.hip}.o
TL=$(python3 -c "import os,torch;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
objs=$(ls build/dvie/*.o | grep -v "/${f%.hip}.o$")
g++ -shared -fPIC -o $out $objs $tmp/${f%.hip}.o -Wl,--no-as-needed -L$TL -l:libamdhip64.so -Wl,-rpath,$TL -Wl,-z,defs
rm -rf $tmp
echo "built $out ($f at $rev)"
