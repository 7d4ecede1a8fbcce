for a in 0 1 2 4 8 15; do echo "abl $a"; ORBFE_OCT_ABL=$a timeout -k 10 100 python tools/octree_profile.py --pairs 128 2>&1 | grep "level [03]" || exit 1; done
