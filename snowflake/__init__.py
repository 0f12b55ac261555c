"""``snowflake`` alias package: ``import snowflake.connector`` resolves to the local Snowflake
warehouse stand-in (hops_examples_amd.snowflake; reference hsfs/snowflake/python.ipynb:51-75)."""
