# same-box A/B of whole steps (encode+decode, HIP-event kernel times): the in-tree library
# against tools/_abl<X>/libdc_core.so, interleaved runs. bash tools/gpu_ab_step.sh X [CFG] [STAGE]
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  echo "tree:"; timeout -k 10 200 python -u tools/kern_ab.py --stage ${3:-step} --option decode_static_pct --values 60 --cfg ${2:-C2} --rounds 3 || exit 1
  echo "abl$1:"; DC_CORE_LIB=$PWD/tools/_abl$1/libdc_core.so timeout -k 10 200 python -u tools/kern_ab.py --stage ${3:-step} --option decode_static_pct --values 60 --cfg ${2:-C2} --rounds 3 || exit 1
done
