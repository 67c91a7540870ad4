import sys; sys.path.insert(0, '.')
import bench
print(bench.hbm_probe())
print(bench.hbm_probe(nbytes=1 << 31))
