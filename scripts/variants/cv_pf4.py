PFD = 4
exec(open("/root/repo/scripts/variants/cv_pf.py").read())
