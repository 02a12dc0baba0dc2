set -e
TAG=r03_nt REPS=2 VARIANTS="tree:2:0:0 nt1:2:0:0 nt2:2:0:0 nt3:2:0:0" bash tools/gpu_relax_ab.sh
