# standalone: which memset nodes lose their ordering in a packet-captured graph on a non-blocking stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
B=stereoalgorithms_amd/bin
LOG=gpurun_out/memset_repro.log
: > $LOG
for nb in "--nonblocking" ""; do
  for z in "8 8" "8 0" "9600 0" "9600 256" "24 8" "4096 4" "65536 0"; do
    set -- $z
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 5 60 $B/overlap_repro --reps 100 $nb --memset-bytes $1 --memset-offset $2 --kernels 120 >> $LOG 2>&1
    r=$?; [ $r -gt 1 ] && { echo "rc=$r" >> $LOG; cat $LOG; exit $r; }
  done
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 5 60 $B/overlap_repro --reps 100 --nonblocking --memset-bytes 8 --memset-offset 8 --kernels 120 >> $LOG 2>&1
r=$?; [ $r -gt 1 ] && exit $r
cat $LOG
