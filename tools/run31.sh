set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r31; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -i -o "[A-Za-z0-9_]*\(UTCL\|TLB\|UTC\)[A-Za-z0-9_]*" $O/avail.txt | sort -u > $O/tlb.txt || true
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt -o kt -- python3 tools/sweep_part.py w2_4l_3 w2_4l_3//128 w2_4l_3 > $O/c2.log 2>&1 || { echo "c2 failed"; tail $O/c2.log; exit 1; }
grep probe $O/c2.log | cut -c1-200; python3 tools/trace_split.py $O/kt base packed8 base
wc -l $O/tlb.txt; head -40 $O/tlb.txt
