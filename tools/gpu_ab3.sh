# same-box A/B/C of one stage over several configs: in-tree library vs tools/_abl<X> libraries
#   bash tools/gpu_ab3.sh "S T" "C2:2 C4:2" encode
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in $2; do
  c=${cfg%%:*}; nary=${cfg##*:}
  for r in 1 2; do
    echo "$c tree:"; timeout -k 10 200 python -u tools/kern_ab.py --stage ${3:-encode} --option decode_static_pct --values 60 --cfg $c --nary $nary --rounds 3 || exit 1
    for x in $1; do
      echo "$c abl$x:"; DC_CORE_LIB=$PWD/tools/_abl$x/libdc_core.so timeout -k 10 200 python -u tools/kern_ab.py --stage ${3:-encode} --option decode_static_pct --values 60 --cfg $c --nary $nary --rounds 3 || exit 1
    done
  done
done
