# pack/decode ablation libraries (tools/_ablN, built by tools/diag_build.sh _ablN -DDC_ABL_...) timed
# against the in-tree library on one stage: bash tools/gpu_abl.sh STAGE "1 2" [CFG]
set -o pipefail
cd $GRAFT_REPO_ROOT
echo "base:"; timeout -k 10 200 python -u tools/kern_ab.py --stage $1 --option decode_static_pct --values 60 --cfg ${3:-C2} --rounds 3 || exit 1
for v in $2; do
  echo "abl$v:"; DC_CORE_LIB=$PWD/tools/_abl$v/libdc_core.so timeout -k 10 200 python -u tools/kern_ab.py --stage $1 --option decode_static_pct --values 60 --cfg ${3:-C2} --rounds 3 || exit 1
done
