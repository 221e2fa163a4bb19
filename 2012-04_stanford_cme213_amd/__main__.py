"""``python -m cme213x <command> [args]`` -- the reference's programs."""
import sys

from .drivers import final, hw1, hw2_hw5, hw3, hw4, studies

COMMANDS = {
    "cipher": hw1.cipher_main,
    "pagerank": hw1.pagerank_main,
    "heat2d": hw2_hw5.heat2d_main,
    "heat2d_mpi": hw2_hw5.heat2d_mpi_main,
    "create_cipher": hw3.create_cipher_main,
    "solve_cipher": hw3.solve_cipher_main,
    "radixsort": hw4.radixsort_main,
    "mergesort": hw4.mergesort_main,
    "fp": final.fp_main,
    "checker": final.checker_main,
    "readmm": final.readmm_main,
    "genfp": final.genfp_main,
    "occupancy": studies.occupancy_main,
    "study": studies.study_main,
}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in COMMANDS:
        print("usage: python -m cme213x <command> [args]\ncommands: " + ", ".join(sorted(COMMANDS)))
        return 1
    return int(COMMANDS[argv[0]](argv[1:]) or 0)


if __name__ == "__main__":
    sys.exit(main())
