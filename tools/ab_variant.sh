#!/bin/bash
# An A/B build of libefeshash from a PATCHED COPY of the sources (the product sources stay the one
# build): tools/ab_variant.sh NAME 'sed-expression' [file under efes_amd/csrc, default efes_kernels.hip]
# -> efes_amd/lib/ab/libefeshash_NAME.so, loaded by bench.py through EFES_LIB_OVERRIDE.  Fails when
# the expression changes nothing.  An expression "git:REV" takes the file as of git revision REV
# instead (an A/B of a rewritten kernel against its predecessor), "file:PATH" the file at PATH.
set -e
cd "$(dirname "$0")/.."
NAME=$1; EXPR=$2; FILE=${3:-efes_kernels.hip}
D=/tmp/efes_ab_$NAME
rm -rf "$D"; mkdir -p "$D/efes_amd" efes_amd/lib/ab
cp -r efes_amd/csrc "$D/efes_amd/"; cp -r include "$D/"
case "$EXPR" in
  git:*) git show "${EXPR#git:}:efes_amd/csrc/$FILE" > "$D/efes_amd/csrc/$FILE" ;;
  file:*) cp "${EXPR#file:}" "$D/efes_amd/csrc/$FILE" ;;
  *) sed -i "$EXPR" "$D/efes_amd/csrc/$FILE" ;;
esac
if cmp -s "$D/efes_amd/csrc/$FILE" "efes_amd/csrc/$FILE"; then echo "ab_variant $NAME: no change" >&2; exit 1; fi
diff -u "efes_amd/csrc/$FILE" "$D/efes_amd/csrc/$FILE" > "efes_amd/lib/ab/$NAME.diff" || true
${HIPCC:-/opt/rocm/bin/hipcc} --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I "$D/include" \
  -o "efes_amd/lib/ab/libefeshash_$NAME.so" "$D"/efes_amd/csrc/*.hip "$D"/efes_amd/csrc/*.cpp
echo "efes_amd/lib/ab/libefeshash_$NAME.so"
