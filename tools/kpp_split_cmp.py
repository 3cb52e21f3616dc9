import sys; sys.argv=['x']
sys.path.insert(0,'tools')
import micro_kpp as M
for (n, dim, k) in [(6040, 64, 604), (3706, 64, 371), (17730, 64, 1773), (40000, 47, 196), (200000, 47, 196)]:
    M.run(n, dim, k, 2, check=False)
