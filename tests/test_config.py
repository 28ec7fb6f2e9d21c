"""run.conf parser (C++), mirroring the reference's libconfig keys (run.conf:1-23, config.c:4-42)."""
import os

import pytest

REF_STYLE = """
application:
{
	NX = 128;
	NY = 128;
	NZ = 65; #Points in physical space are 2*NZ+2
	input:
	{
 		G = "-";
		DDV = "-";
		UMEAN = "-";
		# G = "/drive1/x/G.h5";
	};
	output:
	{
		G = "/tmp/G.01.h5";
		DDV = "/tmp/ddV.01.h5";
		UMEAN = "/tmp/Umean2.bin";
	};
	path = "/tmp/out/";
};
"""


def test_reference_keys(native):
    c = native.Config.from_string(REF_STYLE)
    assert (c.NX, c.NY, c.NZ) == (128, 128, 65)
    assert c.nzp == 128
    assert c.in_G == "-" and c.in_DDV == "-" and c.in_UMEAN == "-"
    assert c.out_G == "/tmp/G.01.h5" and c.out_UMEAN == "/tmp/Umean2.bin"
    assert c.path == "/tmp/out/"
    # reference constants as defaults (channel.h:50-62, RK3.c:68, 124)
    assert c.Re == 3250.0 and c.Q == 1.8 and c.cfl == 0.5 and c.nsteps == 30000 and c.stats_every == 10


def test_overrides_and_roundtrip(native):
    c = native.Config.from_string(REF_STYLE, ["Re=5000", "nsteps=10", 'precision="fp64"', "NY=129"])
    assert c.Re == 5000.0 and c.nsteps == 10 and c.precision == "fp64" and c.NY == 129
    c2 = native.Config.from_string(c.to_string())
    for k in ["NX", "NY", "NZ", "Re", "Q", "LX", "LZ", "nsteps", "cfl", "precision", "path", "out_G", "seed", "ic"]:
        assert getattr(c2, k) == getattr(c, k), k


def test_comments_and_toplevel_keys(native):
    c = native.Config.from_string("""
        /* block comment */
        NX = 64; // line comment
        NY = 65;
        NZ = 33;
        Re = 1e3;
        health_check = false;
    """)
    assert (c.NX, c.NY, c.NZ, c.Re, c.health_check) == (64, 65, 33, 1000.0, False)


def test_file_and_example(native):
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    c = native.Config.from_file(os.path.join(here, "configs", "run.conf"))
    assert c.NX == 128 and c.nsteps == 100 and c.out_G == "G.h5"


@pytest.mark.parametrize("bad", ["NX = 100; NY = 33; NZ = 17;",      # NX not m*2^k (m = 1, 3, ..., 15)
                                 "NX = 272; NY = 33; NZ = 17;",      # 17*2^k
                                 "NX = 2304; NY = 33; NZ = 17;",     # 9*2^k above 2048
                                 "NX = 64; NY = 33; NZ = 16;",       # 2NZ-2 = 30 likewise
                                 "NX = 24; NY = 33; NZ = 17;",       # 3*2^k below 48
                                 "NX = 3072; NY = 33; NZ = 17;",     # above the largest kernel
                                 "NX = 64; NY = 3; NZ = 17;",        # NY too small
                                 "NX = 64; NY = 33; NZ = 17; precision = \"bf16\";",
                                 "NX = 64 NY = 33;",                 # syntax
                                 "application: { NX = 64;"])         # unterminated group
def test_invalid(native, bad):
    with pytest.raises(RuntimeError):
        native.Config.from_string(bad)


@pytest.mark.parametrize("nx,nz", [(96, 97), (192, 49), (384, 193), (768, 385), (1536, 769), (80, 81), (1280, 641),
                                   (48, 25), (2048, 1025), (112, 73), (1792, 481), (576, 289), (1152, 577),
                                   (960, 121), (1920, 961), (176, 89), (1408, 705), (208, 105), (1664, 833)])
def test_non_power_of_two_lengths(native, nx, nz):
    """Grids of the form m*2^k, m = 3, 5, 7, 9, 11, 13, 15 (cuFFT plans of any length in the reference,
    fft.c:17-23)."""
    c = native.Config.from_string(f"NX = {nx}; NY = 33; NZ = {nz};")
    assert c.NX == nx and c.NZ == nz


def test_input_files_imply_file_ic(native):
    c = native.Config.from_string('NX=32; NY=33; NZ=17; input: { G = "g.h5"; DDV = "d.h5"; };')
    assert c.ic == "file"


def test_failure_and_observability_keys(native):
    c = native.Config.from_string('NX=32; NY=33; NZ=17; on_nan = "rollback"; health_every = 5; snapshot_every = 20;'
                                  ' max_rollbacks = 2; rollback_cfl_factor = 0.25; spectra_every = 50;'
                                  ' spectra_planes = "16, 3"; log_json = "run.jsonl";')
    assert (c.on_nan, c.health_every, c.snapshot_every, c.max_rollbacks) == ("rollback", 5, 20, 2)
    assert c.rollback_cfl_factor == 0.25 and c.spectra_every == 50 and c.spectra_planes == "16, 3"
    assert c.log_json == "run.jsonl"
    again = native.Config.from_string(c.to_string())
    assert again.on_nan == "rollback" and again.spectra_planes == "16, 3"
    for bad in ['on_nan = "retry";', 'spectra_planes = "40";', 'spectra_planes = "a";', "health_every = 0;"]:
        with pytest.raises(RuntimeError):
            native.Config.from_string("NX=32; NY=33; NZ=17; " + bad)
