for x in 0 0x10000 0x40000 0x20000 0x50000 0x70000; do
  echo "xopts=$x $(timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --xopts $x 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*')"
done
