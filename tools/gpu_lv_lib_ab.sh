set -u
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2 3; do for l in tools/bin/var/old.so kan-odes_amd/kanode/libkanode.so; do
  echo "$l $(KANODE_LIB=$PWD/$l timeout -k 10 120 python -u tools/lv_ab.py 2>&1 | tail -n 1)" || exit 3
done; done
