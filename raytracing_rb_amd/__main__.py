"""CLI counterpart of src/main.rb:

    python -m raytracing_rb_amd <s|N> <out.png> <world.yml> <camera.yml> [--seed S] [--device D]

``s`` renders on one GPU (Camera#render_sync); ``N`` splits the frame over N
GPU workers (Camera#render_fork).  The reference seeds Random with 1
(main.rb:10); here the seed keys the counter RNG.
"""

import sys


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    seed, device = 1, 0
    if "--seed" in argv:
        i = argv.index("--seed")
        seed = int(argv[i + 1])
        del argv[i:i + 2]
    if "--device" in argv:
        i = argv.index("--device")
        device = int(argv[i + 1])
        del argv[i:i + 2]
    if len(argv) != 4:
        print("parameter error")                      # main.rb:5-8
        return 1
    mode, out_file, world_file, camera_file = argv
    from .api import Camera, World
    world = World(world_file)
    camera = Camera(world, camera_file, device=device, seed=seed)
    if mode == "s":
        camera.render_sync(out_file)
    else:
        camera.render_fork(out_file, int(mode))
    return 0


if __name__ == "__main__":
    sys.exit(main())
