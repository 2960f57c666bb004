set -u
tools/gpu_session.sh pytest smoke || exit $?
tools/ab.sh "base:-:--steps 20 --warmup 5" "nopf:MSBFS_LIB=abl/nopf/libmsbfs.so:--steps 20 --warmup 5" "pf2:MSBFS_LIB=abl/pf2/libmsbfs.so:--steps 20 --warmup 5" "base2:-:--steps 20 --warmup 5" || exit $?
A="--steps 1 --warmup 0 --verify 0"
specs=("kbase:-:$A")
for v in 1 2 4 6 8 16 32; do specs+=("ts$v:MSBFS_LIB=abl/ts$v/libmsbfs.so:$A"); done
tools/kab.sh "${specs[@]}" || exit $?
tools/gpu_session.sh trace26
