#!/usr/bin/env bash
# Round-3 A/B 5: AllegroHand in the compact layout with 21 contacts and 8 LDS link slots vs the dense 12-contact list
AB_ROUNDS=2 bash tools/ab_variants.sh allegro_hand product libhandarm_hip_ahc21k8.so > gpurun_out/ab_ahc21k8.txt 2>&1
cp gpurun_out/ab_libhandarm_hip_ahc21k8_2.json gpurun_out/ab_ahc21k8.json
