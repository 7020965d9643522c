# single-frame CLAHE apply split sweep (tools/clahe_micro.py), one box
for v in default 64 128 256 512 1024; do
  if [ $v = default ]; then E=""; else E="GVX_CLAHE_APPLY_WG=$v"; fi
  env $E timeout -k 10 120 python3 tools/clahe_micro.py 5 2>&1 | grep -E "single|synthetic"
done
