#!/bin/bash
# conv2 forward A/B across library builds: tools/ab/conv2f_ab.py's ring timing with the in-tree
# library and each of tools/ab/$ALTS (diagnostic variants).
cd ${GRAFT_REPO_ROOT:-/root/repo}
L=a2cat-vn-pytorch_amd/vnav/_lib/libvnav.so
cp $L /tmp/new.so
for v in new $ALTS new; do
  if [ $v = new ]; then cp /tmp/new.so $L; else cp tools/ab/$v $L; fi
  echo "$v: $(timeout -k 10 200 python tools/ab/conv2f_ab.py 4096 10 2>/dev/null | tail -1)"
done
cp /tmp/new.so $L
