# Round 3, GPU call ao: where the layout plan's time goes (phase-stop study builds), kernel
# durations from rocprofv3 --stats.
set -eu
O=gpurun_out/r03ao
mkdir -p $O
export TMPDIR=/tmp
for v in base plan1 plan2 plan3; do
  if [ $v = base ]; then L=""; else L="$GRAFT_REPO_ROOT/tools/with_lib.py $GRAFT_REPO_ROOT/tools/ab/libfdx_$v.so"; fi
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/$v -- python3 $L $GRAFT_REPO_ROOT/tools/plan_probe.py > $GRAFT_REPO_ROOT/$O/$v.log 2>&1
  cd $GRAFT_REPO_ROOT
  echo "$v $(cat $O/$v.log | tail -1)"
  grep -h "k_layout_plan_small" $O/$v/*/*_kernel_stats.csv | cut -d, -f1-4
done
echo r03ao done
