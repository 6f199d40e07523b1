# r06: same-box A/B of (old lib, committed table) vs (lib with configs 26-28, table with the K <= 64
# ResNet shapes re-timed): ResNet micro, config-2 bench x4, config-5 bench x2
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=t5-resnet-vqa_amd/lib/libvqa_hip.so; T=t5-resnet-vqa_amd/tuning/gemm_gfx950.json
cp $T gpurun_out/tune_committed.json
A="gpurun_ab/lib_r06_epi_keep.so gpurun_out/tune_committed.json"
B="gpurun_ab/lib_r06_k64.so gpurun_ab/tune_k64_merged.json"
n=0
for pair in "$A" "$B"; do
  set -- $pair; cp $1 $L; cp $2 $T; n=$((n+1))
  timeout -k 10 300 python tools/res_micro.py > gpurun_out/s14_res_$n.txt 2>&1 || { echo MICROFAIL; tail -5 gpurun_out/s14_res_$n.txt; exit 1; }
  echo "res [$1]" $(grep -E "^ +[0-9]+ gemm M= 200704 N=  (256|64) K=   64" gpurun_out/s14_res_$n.txt | awk '{print $11}' | tr '\n' ' ') $(tail -1 gpurun_out/s14_res_$n.txt)
done
i=0
for rep in 1 2 3 4; do
  for pair in "$A" "$B"; do
    set -- $pair; cp $1 $L; cp $2 $T; i=$((i+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s14_ab_$i.json 2> gpurun_out/s14_ab.err || { echo BENCHFAIL; tail -20 gpurun_out/s14_ab.err; exit 1; }
    echo "[$1]" $(python -c "import json;d=json.load(open('gpurun_out/s14_ab_$i.json'));print(d['value'], d['ms_per_step'])")
  done
done
for rep in 1 2; do
  for pair in "$A" "$B"; do
    set -- $pair; cp $1 $L; cp $2 $T
    timeout -k 10 300 python bench.py --config5 --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s14_c5.json 2> gpurun_out/s14_ab.err || { echo C5FAIL; tail -20 gpurun_out/s14_ab.err; exit 1; }
    echo "c5 [$1]" $(python -c "import json;d=json.load(open('gpurun_out/s14_c5.json'));print(d['value'], d['ms_per_step'])")
  done
done
cp gpurun_out/tune_committed.json $T
