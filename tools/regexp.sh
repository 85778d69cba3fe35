for r in 0 65536 24576; do
  if [ $r = 0 ]; then unset ENET_RC_REGION; else export ENET_RC_REGION=$r; fi
  echo "region $r"; ENET_RC_DEBUG=1 timeout -k 10 200 python tools/abx.py A --workload c2 --rounds 8 2>&1 | grep -v amdgpu.ids || exit 1
  ENET_RC_DEBUG=1 timeout -k 10 200 python tools/abx.py A --workload c3 --rounds 4 2>&1 | grep -v amdgpu.ids || exit 1
done
