"""Client IP -> region (reference services/geo.py:11-217).

Offline first: private/unknown addresses map to the default region and a
first-octet table covers the common public ranges; network lookups
(ip-api.com then ipinfo.io) are opt-in via ``settings.geo_lookup_enabled``
and cached for an hour.
"""
from __future__ import annotations

import ipaddress
import logging
import time
from typing import Dict, Optional, Tuple

logger = logging.getLogger(__name__)

DEFAULT_REGION = "asia-east"

REGION_NAMES = {
    "asia-east": "东亚 (East Asia)", "asia-south": "南亚/东南亚 (South & Southeast Asia)",
    "europe-west": "西欧 (Western Europe)", "europe-east": "东欧 (Eastern Europe)",
    "america-north": "北美 (North America)", "america-south": "南美 (South America)",
    "oceania": "大洋洲 (Oceania)",
}

COUNTRY_TO_REGION = {
    **{c: "asia-east" for c in ("CN", "JP", "KR", "TW", "HK", "MO", "MN")},
    **{c: "asia-south" for c in ("IN", "SG", "TH", "VN", "MY", "ID", "PH", "BD", "PK", "LK", "NP")},
    **{c: "europe-west" for c in ("GB", "DE", "FR", "NL", "BE", "ES", "PT", "IT", "IE", "CH", "AT", "SE", "NO",
                                  "DK", "FI", "LU", "IS")},
    **{c: "europe-east" for c in ("RU", "PL", "UA", "CZ", "RO", "HU", "BG", "BY", "SK", "LT", "LV", "EE", "TR")},
    **{c: "america-north" for c in ("US", "CA", "MX")},
    **{c: "america-south" for c in ("BR", "AR", "CL", "CO", "PE", "VE", "EC", "UY", "PY", "BO")},
    **{c: "oceania" for c in ("AU", "NZ", "FJ", "PG")},
}

# coarse first-octet allocation table (RIR blocks / large carriers)
_PREFIX_REGION = {
    2: "europe-west", 3: "america-north", 4: "america-north", 5: "europe-west", 8: "america-north",
    13: "america-north", 14: "asia-east", 18: "america-north", 23: "america-north", 27: "asia-east",
    31: "europe-west", 36: "asia-east", 37: "europe-west", 39: "asia-east", 42: "asia-east", 43: "asia-south",
    46: "europe-east", 49: "asia-east", 52: "america-north", 54: "america-north", 58: "asia-east",
    59: "asia-east", 60: "asia-east", 61: "asia-east", 62: "europe-west", 77: "europe-east", 78: "europe-west",
    80: "europe-west", 81: "europe-west", 82: "europe-west", 83: "europe-west", 84: "europe-west",
    85: "europe-west", 86: "europe-west", 87: "europe-west", 88: "europe-west", 89: "europe-west",
    90: "europe-west", 91: "europe-west", 92: "europe-west", 93: "europe-west", 94: "europe-west",
    95: "europe-east", 101: "asia-east", 103: "asia-south", 106: "asia-east", 110: "asia-east",
    111: "asia-east", 112: "asia-east", 113: "asia-east", 114: "asia-east", 115: "asia-east",
    116: "asia-east", 117: "asia-east", 118: "asia-east", 119: "asia-east", 120: "asia-east",
    121: "asia-east", 122: "asia-east", 123: "asia-east", 124: "asia-east", 125: "asia-east",
    175: "asia-east", 177: "america-south", 179: "america-south", 180: "asia-east", 181: "america-south",
    182: "asia-east", 183: "asia-east", 186: "america-south", 187: "america-south", 189: "america-south",
    190: "america-south", 191: "america-south", 200: "america-south", 201: "america-south",
    202: "asia-east", 203: "oceania", 210: "asia-east", 211: "asia-east", 218: "asia-east",
    219: "asia-east", 220: "asia-east", 221: "asia-east", 222: "asia-east", 223: "asia-east",
}

_cache: Dict[str, Tuple[str, float]] = {}
_CACHE_TTL = 3600.0
_CACHE_MAX = 10000
_client = None


def get_region_name(region: str) -> str:
    return REGION_NAMES.get(region, region)


def get_region_info(region: str) -> Dict[str, str]:
    return {"code": region, "name": get_region_name(region)}


def _is_private(ip: str) -> bool:
    if ip in ("localhost", "", "testclient"):
        return True
    try:
        a = ipaddress.ip_address(ip)
        return a.is_private or a.is_loopback or a.is_link_local or a.is_reserved
    except ValueError:
        return True


def _prefix_region(ip: str) -> Optional[str]:
    try:
        a = ipaddress.ip_address(ip)
    except ValueError:
        return None
    if a.version == 4:
        return _PREFIX_REGION.get(int(str(a).split(".")[0]))
    return None


async def _lookup_network(ip: str) -> Optional[str]:
    global _client
    try:
        import httpx
        if _client is None:
            _client = httpx.AsyncClient(timeout=2.0)
        r = await _client.get(f"http://ip-api.com/json/{ip}?fields=countryCode")
        cc = r.json().get("countryCode") if r.status_code == 200 else None
        if not cc:
            r = await _client.get(f"https://ipinfo.io/{ip}/json")
            cc = r.json().get("country") if r.status_code == 200 else None
        return COUNTRY_TO_REGION.get(cc or "")
    except Exception as e:
        logger.debug("geo lookup failed for %s: %s", ip, e)
        return None


async def detect_client_region(ip: Optional[str]) -> str:
    if not ip or _is_private(ip):
        return DEFAULT_REGION
    hit = _cache.get(ip)
    if hit and time.time() - hit[1] < _CACHE_TTL:
        return hit[0]
    region = _prefix_region(ip)
    if region is None:
        try:
            from app.config import settings
            net = settings.geo_lookup_enabled
        except Exception:
            net = False
        if net:
            region = await _lookup_network(ip)
    region = region or DEFAULT_REGION
    if len(_cache) >= _CACHE_MAX:
        _cache.pop(next(iter(_cache)))
    _cache[ip] = (region, time.time())
    return region


async def cleanup_resources() -> None:
    global _client
    if _client is not None:
        await _client.aclose()
        _client = None
