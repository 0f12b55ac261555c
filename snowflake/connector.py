"""``snowflake.connector`` -> hops_examples_amd.snowflake (connect, DB-API cursor, write_pandas)."""
from hops_examples_amd.snowflake import (Error, ProgrammingError, SnowflakeConnection, SnowflakeCursor,  # noqa: F401
                                         connect, paramstyle, write_pandas)
