exec(open("/root/repo/scripts/variants/ft_hA.py").read())
exec(open("/root/repo/scripts/variants/ft_wg.py").read())
