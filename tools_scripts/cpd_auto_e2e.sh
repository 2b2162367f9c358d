# One GPU call: bin/make_cpd_auto end to end (read, plan, build, copy out,
# write bucket files) on a synthetic graph, sequential (--no-pipeline) vs the
# overlapped writer; the files of both runs are compared byte for byte.
#   bash tools_scripts/cpd_auto_e2e.sh WIDTH KEY   (div KEY, worker 0 of KEY)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
WIDTH=${1:-300}
KEY=${2:-8}
T=$(mktemp -d /tmp/cpde2e.XXXX)
trap 'rm -rf $T' EXIT
mkdir -p $O
$R/bin/gen_synth --width $WIDTH --height $WIDTH --seed 1 --out $T/g --queries 10 > /dev/null
A="--input $T/g.xy --partmethod div --partkey $KEY --workerid 0 --maxworker $KEY --device 0 --plan $T/g.plan"
timeout -k 10 300 $R/bin/make_cpd_auto $A --outdir $T/warm --no-pipeline > /dev/null
rm -rf $T/warm
timeout -k 10 300 $R/bin/make_cpd_auto $A --outdir $T/seq --no-pipeline | tee $O/e2e_seq_$WIDTH.log
timeout -k 10 300 $R/bin/make_cpd_auto $A --outdir $T/pipe | tee $O/e2e_pipe_$WIDTH.log
du -sh $T/seq
cmp <(cat $T/seq/*.cpd | md5sum) <(cat $T/pipe/*.cpd | md5sum) && echo files-identical
