"""Pack a DeepMimic character file + motion clip into the npz bundle that
`ReferenceMotion.from_bundle` loads (amp_extensions_amd/data/humanoid3d_spinkick.npz).

The bundle holds the data only (the character JSON text and the clip frames); run here, where
the reference's data files exist:

  python tools/pack_motion.py /root/reference/deepmimic/deepmimic/data/characters/humanoid3d.txt \
      /root/reference/deepmimic/deepmimic/data/motions/humanoid3d_spinkick.txt \
      amp_extensions_amd/data/humanoid3d_spinkick.npz
"""
import json
import sys

import numpy as np


def pack(character_path: str, motion_path: str, out_path: str) -> None:
    with open(character_path) as f:
        character = json.load(f)
    with open(motion_path) as f:
        motion = json.load(f)
    np.savez_compressed(out_path, character_json=np.array(json.dumps(character)),
                        frames=np.asarray(motion["Frames"], dtype=np.float64),
                        loop=np.array(str(motion.get("Loop", "none"))))


if __name__ == "__main__":
    pack(*sys.argv[1:4])
