# Build liborbx.so from the sources of git revision REV into
# orbslam2commentedbyxcm_amd/_ab/liborbx_TAG.so (A/B against the working tree).
# usage: bash tools/build_rev.sh TAG [REV]
set -e
TAG=$1; REV=${2:-HEAD}
R=$(pwd); T=$(mktemp -d)
git archive "$REV" orbslam2commentedbyxcm_amd/csrc include | tar -x -C "$T"
mkdir -p "$R/orbslam2commentedbyxcm_amd/_ab/obj_$TAG"
F="-O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt --offload-arch=gfx950 -I$T/include -I$T/orbslam2commentedbyxcm_amd/csrc"
objs=""
for s in "$T"/orbslam2commentedbyxcm_amd/csrc/*.hip "$T"/orbslam2commentedbyxcm_amd/csrc/*.cpp; do
  o="$R/orbslam2commentedbyxcm_amd/_ab/obj_$TAG/$(basename $s).o"
  /opt/rocm/bin/hipcc $F -c "$s" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$R/orbslam2commentedbyxcm_amd/_ab/liborbx_$TAG.so" $objs
rm -rf "$T"
echo "$R/orbslam2commentedbyxcm_amd/_ab/liborbx_$TAG.so"
