import numpy as np, sys
sys.path.insert(0, '.')
from deequ_amd.table import Table
from deequ_amd import engine
n = 65537
rng = np.random.default_rng(n)
for name, arr in [("l", rng.integers(-50, 50, n).astype(np.int64)), ("u", rng.permutation(n).astype(np.int64)),
                  ("b", rng.integers(0, 2, n).astype(np.bool_))]:
    t = Table.from_arrays({name: arr})
    try:
        ft = engine.frequencies(t, [name])
        print(name, ft.summary())
    except Exception as e:
        print(name, "ERR", e)
