"""The reference's configuration options that change its records
(config_generator.cc:28-44, global_config.h:350-365, libmerc_config
libmerc.h:109-154) are REFUSED -- by mfp_init / mfp_parse_filter and by the
libmerc shim's mercury_init, with the reason in the error text -- instead of
being accepted and ignored; options that leave this path's records unchanged
are accepted; report_os is honoured from either source.  CPU only (parsing).
"""
import ctypes

import pytest

import mercury_amd
from tests.test_json import _LibmercConfig

BASE = "select=tls,http"

REFUSED = ["metadata", "metadata=1", "certs-json", "raw-features=tls", "raw-features=all", "raw-features=smb,stun",
           "crypto-assess", "crypto-assess=quantum_safe", "network-behavioral-detections", "exposed-creds",
           "http-headers=all", "http-body-max=100", "nonselected-tcp-data", "nonselected-udp-data=1",
           "quic-trial-decryption", "minimize-ram", "fp_proc_threshold=0.5", "proc_dst_threshold=0.1", "stats"]
ACCEPTED = ["metadata=0", "certs-json=0", "dns-json", "stats-blocking", "max_stats_entries=100",
            "raw-features=smb,bittorrent", "raw-features=none", "http-body-max=0", "fp_proc_threshold=0",
            "nonselected-tcp-data=0", "report_os", "report_os=0", "reassembly"]


@pytest.mark.parametrize("opt", REFUSED)
def test_output_changing_option_refused(opt):
    with pytest.raises(mercury_amd.api.MercuryAmdError) as e:
        mercury_amd.parse_filter(f"{BASE};{opt}")
    assert opt.split("=")[0] in str(e.value)


@pytest.mark.parametrize("opt", ACCEPTED)
def test_option_without_effect_accepted(opt):
    sel, fmt = mercury_amd.parse_filter(f"{BASE};{opt}")
    assert sel == mercury_amd.parse_filter("tls,http")[0] != 0


def _init(**fields):
    lib = mercury_amd.load_library()
    lib.mercury_init.restype = ctypes.c_void_p
    lib.mercury_init.argtypes = [ctypes.POINTER(_LibmercConfig), ctypes.c_int]
    lib.mercury_finalize.argtypes = [ctypes.c_void_p]
    cfg = _LibmercConfig()
    cfg.packet_filter_cfg = fields.pop("filt", "tls,http").encode()
    for k, v in fields.items():
        setattr(cfg, k, v)
    mc = lib.mercury_init(ctypes.byref(cfg), 0)
    if mc:
        lib.mercury_finalize(mc)
    return bool(mc)


@pytest.mark.parametrize("field,value", [("metadata_output", True), ("certs_json_output", True),
                                         ("output_tcp_initial_data", True), ("output_udp_initial_data", True),
                                         ("do_stats", True), ("fp_proc_threshold", 0.25),
                                         ("proc_dst_threshold", 0.25)])
def test_libmerc_config_field_refused(field, value):
    """mercury_init returns NULL for a libmerc_config that asks for records
    this path does not write (libmerc.cc:92-128 returns NULL on failure)."""
    assert not _init(**{field: value})


def test_libmerc_config_accepted():
    assert _init()
    assert _init(dns_json_output=True)
    assert _init(report_os=True)
    assert not _init(filt="select=tls;metadata")
    assert _init(filt="select=tls;metadata=0;report_os")
