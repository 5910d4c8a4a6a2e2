# C5 decode step: the current tree and oldtree/ (the r02s2 commit), same box
set -o pipefail
for i in 1 2; do
  timeout -k 10 300 python3 tools/wlbench.py c5 10 3 2>&1 | grep ms/step | sed 's/^/new: /'
  timeout -k 10 300 python3 oldtree/tools/wlbench.py c5 10 3 2>&1 | grep -E "ms/step|Error" | sed 's/^/old: /'
done
