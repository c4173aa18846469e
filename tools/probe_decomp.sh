# Decomposition choice at 1024^3 fp64 (virtual ranks on one GPU): per-subdomain
# compute overheads of slab vs block splits for the 2/4/8-GPU shares.
for d in 2x1x1 4x1x1 2x2x1 8x1x1 4x2x1 2x2x2; do
  IFS=x read a b c <<< "$d"; n=$((a*b*c))
  echo "## $d"
  timeout -k 10 120 python bench.py --steps 150 --warmup 15 --virtual-ranks $n --decomp $d --converge-eps 0 || exit 1
done
