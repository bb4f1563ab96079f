# tools/profile_round.sh ROUND WORKLOADS... (on the GPU box): tools/profile.sh for each workload,
# with the kernels that make up its step.  c2 = partitioned headline, c2ord / c3ord = reference order.
R=$1; shift
for w in "$@"; do
  case $w in
    c2)    PMC_KERNEL="slot_split_pipe|probe_walk" bash tools/profile.sh ${R}_c2 --no-other --no-other-workloads --no-scaling-reference --no-cpu || exit 1 ;;
    c2ord) PMC_KERNEL="slot_split_pipe|probe_walk|unsplit_words|emit_ordered" bash tools/profile.sh ${R}_c2ord --path ordered --no-other --no-other-workloads --no-scaling-reference --no-cpu || exit 1 ;;
    c3)    PMC_KERNEL="slot_split_pipe|probe_chain_filt|probe_chain_win|copy_rows_flat" bash tools/profile.sh ${R}_c3 --workload c3 --no-cpu || exit 1 ;;
    c3ord) PMC_KERNEL="slot_split_pipe|probe_chain_filt|chain_words|unsplit_words|emit_ordered|copy_rows_flat" bash tools/profile.sh ${R}_c3ord --workload c3 --path ordered --no-cpu || exit 1 ;;
    c5)    PMC_KERNEL="slot_split_pipe|probe_walk1|probe_walk2|probe_win|gather_payload" bash tools/profile.sh ${R}_c5 --workload c5 --no-cpu || exit 1 ;;
  esac
done
