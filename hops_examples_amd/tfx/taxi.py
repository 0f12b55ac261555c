"""Raw Chicago-taxi trips with the public dataset's column names (synthetic: there is no network for
the BigQuery extract).  Schema and feature roles follow the public TFX taxi example the reference
README points to (README.md:99-112); the model-side constants live in ``models.widedeep``."""
from __future__ import annotations

import numpy as np
import pandas as pd

from ..models.widedeep import (BUCKET_FEATURE_KEYS, CATEGORICAL_FEATURE_KEYS, DENSE_FLOAT_FEATURE_KEYS,  # noqa: F401
                               FEATURE_BUCKET_COUNT, LABEL_KEY, MAX_CATEGORICAL_FEATURE_VALUES, OOV_SIZE,
                               VOCAB_FEATURE_KEYS, VOCAB_SIZE)

FARE_KEY = "fare"
TIP_FRACTION = 0.2  # label: tips > 20 % of the fare ("big tipper")
PAYMENT_TYPES = ["Credit Card", "Cash", "No Charge", "Unknown", "Dispute", "Pcard", "Prcard", "Mobile"]
RAW_COLUMNS = (["trip_start_timestamp"] + DENSE_FLOAT_FEATURE_KEYS + BUCKET_FEATURE_KEYS + VOCAB_FEATURE_KEYS
               + CATEGORICAL_FEATURE_KEYS + [LABEL_KEY])


def synth_raw_trips(n: int, seed: int = 0, missing: float = 0.02, n_companies: int = 1400) -> pd.DataFrame:
    """``n`` raw trips.  Numeric columns carry ~``missing`` NaNs (the real extract has gaps in the
    community areas, census tracts and coordinates), ``company`` has more distinct values than the
    1000-entry vocabulary (so the OOV buckets are exercised) and a heavy-tailed frequency."""
    r = np.random.default_rng(seed)
    ts = r.integers(1_356_998_400, 1_483_228_800, n)  # 2013 .. 2016, seconds
    t = pd.to_datetime(ts, unit="s")
    miles = r.gamma(1.4, 2.5, n).astype(np.float32)
    secs = (miles * r.uniform(150, 420, n) + r.uniform(60, 300, n)).astype(np.float32)
    fare = (3.25 + 2.25 * miles + secs / 36.0 * 0.25 + r.normal(0, 1.0, n)).clip(3.25).astype(np.float32)
    pay = r.choice(len(PAYMENT_TYPES), n, p=[0.52, 0.4, 0.02, 0.02, 0.01, 0.01, 0.01, 0.01])
    comp = np.minimum((n_companies * r.random(n) ** 2.2).astype(np.int64), n_companies - 1)
    plat = r.normal(41.89, 0.05, n).astype(np.float32)
    plon = r.normal(-87.65, 0.04, n).astype(np.float32)
    dlat = (plat + r.normal(0, 0.03, n)).astype(np.float32)
    dlon = (plon + r.normal(0, 0.03, n)).astype(np.float32)
    # tip behaviour: card payers tip, cash tips are rarely recorded; longer trips, later hours tip more
    logit = (np.where(pay == 0, 1.6, -2.5) + 0.08 * miles + 0.03 * (t.hour.to_numpy() - 12)
             - 0.002 * comp + r.normal(0, 0.7, n))
    tips = np.where(1 / (1 + np.exp(-logit)) > r.random(n), fare * r.uniform(0.18, 0.3, n),
                    fare * r.uniform(0.0, 0.1, n)).astype(np.float32)
    df = pd.DataFrame({
        "trip_start_timestamp": ts,
        "trip_miles": miles, "fare": fare, "trip_seconds": secs,
        "pickup_latitude": plat, "pickup_longitude": plon, "dropoff_latitude": dlat, "dropoff_longitude": dlon,
        "payment_type": np.array(PAYMENT_TYPES, dtype=object)[pay],
        "company": np.array([f"{c:04d} - Taxi Co" for c in range(n_companies)], dtype=object)[comp],
        "trip_start_hour": t.hour.to_numpy().astype(np.float32),
        "trip_start_day": t.dayofweek.to_numpy().astype(np.float32) + 1,
        "trip_start_month": t.month.to_numpy().astype(np.float32),
        "pickup_census_tract": r.integers(0, 2000, n).astype(np.float32),
        "dropoff_census_tract": r.integers(0, 2000, n).astype(np.float32),
        "pickup_community_area": r.integers(1, 78, n).astype(np.float32),
        "dropoff_community_area": r.integers(1, 78, n).astype(np.float32),
        LABEL_KEY: tips,
    })
    for c in ["trip_miles", "trip_seconds", "pickup_latitude", "pickup_longitude", "dropoff_latitude",
              "dropoff_longitude", "pickup_census_tract", "dropoff_census_tract", "pickup_community_area",
              "dropoff_community_area"]:
        df.loc[r.random(n) < missing, c] = np.nan
    df.loc[r.random(n) < missing, "company"] = None
    df.loc[r.random(n) < missing / 4, "fare"] = np.nan
    return df
