import os, sys
sys.path.insert(0, 'sfm-mvs-pipeline_amd'); sys.path.insert(0, 'tests')
import numpy as np
from test_gpu_ba import _hard_problem, gpu_solve
p = _hard_problem(0)
for spec in ("0", "1"):
    os.environ["SFMX_BA_SPEC"] = spec
    P, sm, tr = gpu_solve(p, max_num_iterations=40)
    print("spec", spec, {k: sm[k] for k in ("final_cost", "termination_type", "num_successful_steps", "num_unsuccessful_steps", "num_invalid_steps", "final_radius")})
    np.set_printoptions(precision=17, linewidth=200)
    print(tr)
