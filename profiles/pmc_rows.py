"""Print the rows of one kernel from a rocprofv3 --pmc output directory (counter_collection.csv), compactly:
    python profiles/pmc_rows.py <dir> <kernel substring>
One line per (dispatch, counter): kernel, duration ns, counter, value."""
import csv
import glob
import sys

d, key = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            print(f'{r["Kernel_Name"][:60]},{int(r["End_Timestamp"]) - int(r["Start_Timestamp"])},'
                  f'{r["Counter_Name"]},{r["Counter_Value"]}')
