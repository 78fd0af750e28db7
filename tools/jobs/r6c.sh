# round 6: frame-order block shapes (VR_XBLOCK) for the traffic-bound oblique
# frames: baked C1 (plane copy), record C1 (quad brick), entropy C0
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 400 python -u tools/bench_variants.py --variants main --config 1024x8 --baked --cameras C1 --rounds 5 --env '' VR_XBLOCK=2,2 VR_XBLOCK=1,8 VR_XBLOCK=2,4 VR_XBLOCK=4,4 VR_XBLOCK=1,16 VR_XBLOCK=4,8 VR_WG_PER_CU=3 VR_WG_PER_CU=3,VR_XBLOCK=2,2 VR_WG_PER_CU=6,VR_XBLOCK=2,4 > $O/baked_C1_xblock.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --variants main --config 1024x8 --cameras C1 --rounds 4 --env '' VR_XBLOCK=2,2 VR_XBLOCK=1,8 VR_XBLOCK=2,4 VR_XBLOCK=4,4 > $O/rec_C1_xblock.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --variants main --config 1024x8 --cameras C0 --method 3 --rounds 3 --env '' VR_XBLOCK=2,2 VR_XBLOCK=1,8 VR_XBLOCK=2,4 > $O/m3_C0_xblock.log 2>&1 || exit 1
echo ok
